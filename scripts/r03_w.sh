#!/bin/bash
# round 3: tree closed mode with 32-bit per-depth counters for 112 depths (14 workgroups per CU instead of 12): parity + A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TLCG_JIT_DEFINES="TLCG_TREE_LVL32;TLCG_TREE_LV=112" timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_limits.py -m gpu -x -q --timeout 150 --timeout-method thread -k "g9deep or W_ or compaction_times" > gpurun_out/r03w_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r03w_pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python -u scripts/probe.py "base:g9deep" "lv112:g9deep||TLCG_TREE_LVL32;TLCG_TREE_LV=112" "lv32:g9deep||TLCG_TREE_LVL32" "base:g9deep" "lv112:g9deep||TLCG_TREE_LVL32;TLCG_TREE_LV=112" "lv32:g9deep||TLCG_TREE_LVL32" > gpurun_out/r03w_probe.jsonl 2>&1; rc=$?; cut -c1-200 gpurun_out/r03w_probe.jsonl; exit $rc
