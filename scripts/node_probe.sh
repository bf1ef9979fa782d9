#!/bin/bash
# where the time of tlcg_run_node's level loop goes with 8 ranks on one GPU
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TLCG_RANK_TRACE=1 timeout -k 10 300 python -u scripts/node_bench.py 8 > gpurun_out/node8t.log 2>&1; tail -30 gpurun_out/node8t.log
timeout -k 10 300 python -u scripts/exchange_virtual.py 8 > gpurun_out/xv8.log 2>&1; tail -3 gpurun_out/xv8.log
