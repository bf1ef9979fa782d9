#!/bin/bash
# round 3: the tree's store reads in a uniform branch with their own wait (no vmcnt(0) on the frontier-buffer path) vs one merged read
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_tree.py tests/test_gpu_parity.py tests/test_gpu_limits.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03af_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r03af_pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python -u scripts/probe.py "split:g9deep" "merged:g9deep||TLCG_TREE_SPLIT_LOAD=0" "split:g9deep" "merged:g9deep||TLCG_TREE_SPLIT_LOAD=0" "split:g9deep" "merged:g9deep||TLCG_TREE_SPLIT_LOAD=0" > gpurun_out/r03af_probe.jsonl 2>&1; rc=$?; cut -c1-200 gpurun_out/r03af_probe.jsonl; exit $rc
