#!/bin/bash
# round 3: the tree's closed mode storing codes -- parity, A/B against word stores, counters
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_tree.py tests/test_gpu_limits.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r03i_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r03i_pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python -u scripts/probe.py "codes:g9deep" "words:g9deep||TLCG_TREE_CODE_STORE=0" "codes:g9deep" "words:g9deep||TLCG_TREE_CODE_STORE=0" > gpurun_out/r03i_probe.jsonl 2>&1; rc=$?; cut -c1-200 gpurun_out/r03i_probe.jsonl; [ $rc = 0 ] || exit $rc
bash scripts/pmc_kernel.sh "x:g9deep" treec r03_tree_g9deep > gpurun_out/r03i_pmc_tree_g9deep.json; rc=$?; cut -c1-300 gpurun_out/r03i_pmc_tree_g9deep.json; exit $rc
