#!/bin/bash
# round 3: the tree's closed-mode slots displaced by the host's perfect-hash table (one CAS per insert) vs linear probing alone
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_tree.py tests/test_gpu_parity.py tests/test_gpu_limits.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03ag_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r03ag_pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python -u scripts/probe.py "disp:g9deep" "nodisp:g9deep||TLCG_TREE_DISP=0" "disp:g9deep" "nodisp:g9deep||TLCG_TREE_DISP=0" "disp:g9deep" "nodisp:g9deep||TLCG_TREE_DISP=0" > gpurun_out/r03ag_probe.jsonl 2>&1; rc=$?; cut -c1-200 gpurun_out/r03ag_probe.jsonl; exit $rc
