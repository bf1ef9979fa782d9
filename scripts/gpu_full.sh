#!/bin/bash
# round verification: smoke, all -m gpu tests, the default bench + its
# rocprofv3 kernel stats, the per-config baseline table, the 8-rank node bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_round.sh || exit 1
bash scripts/baseline_table.sh || exit 1
timeout -k 10 300 python -u scripts/node_bench.py 8 > gpurun_out/node8.jsonl 2>&1 || exit 1
cat gpurun_out/node8.jsonl
