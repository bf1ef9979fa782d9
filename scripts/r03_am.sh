#!/bin/bash
# round 3: the tree's closed-mode invariants evaluated at expansion (one per step) vs at insert (one per insert call)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_tree.py tests/test_gpu_parity.py tests/test_gpu_limits.py tests/test_gpu_user_inv.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03am_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r03am_pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python -u scripts/probe.py "expand:g9deep" "insert:g9deep||TLCG_TREE_INV_AT_EXPAND=0" "expand:g9deep" "insert:g9deep||TLCG_TREE_INV_AT_EXPAND=0" "expand:g9deep" "insert:g9deep||TLCG_TREE_INV_AT_EXPAND=0" > gpurun_out/r03am_probe.jsonl 2>&1; rc=$?; cut -c1-200 gpurun_out/r03am_probe.jsonl; exit $rc
