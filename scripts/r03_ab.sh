#!/bin/bash
# round 3: tlcg_run_node with contexts created/destroyed by one thread per rank: tests + G9 at 8 virtual ranks
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_partition.py tests/test_gpu_cli.py tests/test_gpu_tree.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r03ab_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r03ab_pytest.log; [ $rc = 0 ] || exit $rc
TLCG_RANK_TRACE=1 timeout -k 10 300 python -u scripts/node_bench.py 8 15 > gpurun_out/r03ab_node8_g9.jsonl 2> gpurun_out/r03ab_node8_g9.trace; rc=$?; cat gpurun_out/r03ab_node8_g9.jsonl; exit $rc
