#!/bin/bash
# round 3: striped counters -- parity of the engines, then the grid sweep again
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_tree.py tests/test_gpu_limits.py tests/test_gpu_random_cfgs.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03c_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r03c_pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 900 python -u scripts/probe.py \
  "m8:m8" "m8g4096:m8|TLCG_COMP_GRID=4096" "m8g8192:m8|TLCG_COMP_GRID=8192" "m8g12288:m8|TLCG_COMP_GRID=12288" "m8g16384:m8|TLCG_COMP_GRID=16384" \
  "sh0:g9:0/8" "sh0g8192:g9:0/8|TLCG_COMP_GRID=8192" "sh0g12288:g9:0/8|TLCG_COMP_GRID=12288" "sh0g16384:g9:0/8|TLCG_COMP_GRID=16384" \
  "g9:g9" "g9g32768:g9|TLCG_COMP_GRID=32768" "g9g131072:g9|TLCG_COMP_GRID=131072" "g9g262144:g9|TLCG_COMP_GRID=262144" \
  "g9deep:g9deep" "g9deepg8192:g9deep|TLCG_TREE_GRID=8192" "g9deepg32768:g9deep|TLCG_TREE_GRID=32768" "g9deepg65536:g9deep|TLCG_TREE_GRID=65536" \
  "p8:p8" "p8g8192:p8|TLCG_TREE_GRID=8192" "p8g32768:p8|TLCG_TREE_GRID=32768" "p8g65536:p8|TLCG_TREE_GRID=65536" \
  > gpurun_out/r03c_probe.jsonl 2>&1; rc=$?; cut -c1-200 gpurun_out/r03c_probe.jsonl; exit $rc
