#!/bin/bash
# where the time of tlcg_run_node's level loop goes with 8 ranks on one GPU,
# and the FPSet access ceilings with the table split by XCD
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TLCG_RANK_TRACE=1 timeout -k 10 300 python -u scripts/node_bench.py 8 > gpurun_out/node8t.log 2>&1; grep -v "^rank [0-9]: 20 levels" gpurun_out/node8t.log | tail -12
grep "^rank 0: 20 levels" gpurun_out/node8t.log
timeout -k 10 120 ./pulsar-tlaplus_amd/bin/fpset_microbench 31 1073741824 0 > gpurun_out/micro.jsonl 2>&1; cat gpurun_out/micro.jsonl
timeout -k 10 300 python -u scripts/comp_variants.py > gpurun_out/cv.log 2>&1; tail -5 gpurun_out/cv.log
