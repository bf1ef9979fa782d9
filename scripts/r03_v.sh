#!/bin/bash
# round 3: pair mode in the Producer tree (A/B + parity with it on)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TLCG_JIT_DEFINES="TLCG_TREE_PAIR_OPEN=1" TLCG_JIT=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_tree.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r03v_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r03v_pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python -u scripts/probe.py "base:p8" "pair:p8||TLCG_TREE_PAIR_OPEN=1" "base:p8" "pair:p8||TLCG_TREE_PAIR_OPEN=1" > gpurun_out/r03v_probe.jsonl 2>&1; rc=$?; cut -c1-200 gpurun_out/r03v_probe.jsonl; exit $rc
