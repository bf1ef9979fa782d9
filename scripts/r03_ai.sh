#!/bin/bash
# round 3: the tree's first CAS outside the probe loop (closed mode, behind the perfect hash) vs inside
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_tree.py tests/test_gpu_parity.py tests/test_gpu_limits.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03ai_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r03ai_pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python -u scripts/probe.py "cas1:g9deep" "loop:g9deep||TLCG_TREE_CAS1=0" "cas1:g9deep" "loop:g9deep||TLCG_TREE_CAS1=0" "cas1:g9deep" "loop:g9deep||TLCG_TREE_CAS1=0" > gpurun_out/r03ai_probe.jsonl 2>&1; rc=$?; cut -c1-200 gpurun_out/r03ai_probe.jsonl; exit $rc
