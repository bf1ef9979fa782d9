#!/bin/bash
# round 3: tree closed mode, pair mode (a narrow depth in one step with one insert) -- parity, A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_tree.py tests/test_gpu_parity.py tests/test_gpu_partition.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r03t_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r03t_pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python -u scripts/probe.py "pair:g9deep" "two:g9deep||TLCG_TREE_PAIR=0" "pair:g9deep" "two:g9deep||TLCG_TREE_PAIR=0" "pair:p8" > gpurun_out/r03t_probe.jsonl 2>&1; rc=$?; cut -c1-200 gpurun_out/r03t_probe.jsonl; exit $rc
