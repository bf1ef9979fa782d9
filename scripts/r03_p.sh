#!/bin/bash
# round 3: component counters folded and reset on the device (parity: every
# component test incl. the K0=32 cascade), then A/B of the successors'
# invariants evaluated before their probes, and the per-check wall overhead
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_partition.py tests/test_gpu_random_cfgs.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r03p_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r03p_pytest.log; [ $rc = 0 ] || exit $rc
PROBE_REPS=6 timeout -k 10 600 python -u scripts/probe.py "base:g9" "spec:g9||TLCG_SPEC_INV=1" "base:g9" "spec:g9||TLCG_SPEC_INV=1" "base:m8" "spec:m8||TLCG_SPEC_INV=1" "sh:g9:0/8" "sh:g9:0/8" > gpurun_out/r03p_probe.jsonl 2>&1; rc=$?; cut -c1-200 gpurun_out/r03p_probe.jsonl; exit $rc
