#!/bin/bash
# round 3: the second successor's queue entry read before the first one's probe (A/B), parity with it on
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TLCG_JIT_DEFINES="TLCG_PREFETCH_Q2=1" TLCG_JIT=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 150 --timeout-method thread -k "component or golden or g9 or m8" > gpurun_out/r03r_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r03r_pytest.log; [ $rc = 0 ] || exit $rc
PROBE_REPS=6 timeout -k 10 600 python -u scripts/probe.py "base:g9" "q2:g9||TLCG_PREFETCH_Q2=1" "base:g9" "q2:g9||TLCG_PREFETCH_Q2=1" "base:m8" "q2:m8||TLCG_PREFETCH_Q2=1" > gpurun_out/r03r_probe.jsonl 2>&1; rc=$?; cut -c1-200 gpurun_out/r03r_probe.jsonl; exit $rc
