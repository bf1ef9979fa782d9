#!/bin/bash
# round 3: tuned slot-hash multipliers (component codes, tree closed mode) -- parity, then A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_tree.py tests/test_gpu_limits.py tests/test_gpu_random_cfgs.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03f_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r03f_pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 900 python -u scripts/probe.py \
  "g9:g9" "g9def:g9|TLCG_TUNE_MULT=0" "g9:g9" "g9def:g9|TLCG_TUNE_MULT=0" \
  "m8:m8" "m8def:m8|TLCG_TUNE_MULT=0" "sh0:g9:0/8" "sh0def:g9:0/8|TLCG_TUNE_MULT=0" \
  "g9deep:g9deep" "g9deepdef:g9deep|TLCG_TUNE_MULT=0" "g9deep:g9deep" "p8:p8" \
  > gpurun_out/r03f_probe.jsonl 2>&1; rc=$?; cut -c1-200 gpurun_out/r03f_probe.jsonl; exit $rc
