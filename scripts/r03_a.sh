#!/bin/bash
# round 3, first call: GPU parity of the changed kernels, then per-config
# kernel times (lane-column LDS A/B, grid caps, 1/8 shares), then counters
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_tree.py tests/test_gpu_limits.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03a_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r03a_pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 900 python -u scripts/probe.py \
  "g9:g9" "g9c0:g9||TLCG_LDS_COLS=0" "g9:g9" "g9c0:g9||TLCG_LDS_COLS=0" \
  "m8:m8" "m8c0:m8||TLCG_LDS_COLS=0" "m8:m8" "m8g3072:m8|TLCG_COMP_GRID=3072" "m8g1536:m8|TLCG_COMP_GRID=1536" "m8g6144:m8|TLCG_COMP_GRID=6144" \
  "sh0:g9:0/8" "sh7:g9:7/8" "sh0g3072:g9:0/8|TLCG_COMP_GRID=3072" "sh0c0:g9:0/8||TLCG_LDS_COLS=0" \
  "g9g3072:g9|TLCG_COMP_GRID=3072" "g9g16384:g9|TLCG_COMP_GRID=16384" \
  "g9deep:g9deep" "p8:p8" > gpurun_out/r03a_probe.jsonl 2>&1; rc=$?; cat gpurun_out/r03a_probe.jsonl | cut -c1-300; [ $rc = 0 ] || exit $rc
bash scripts/pmc_kernel.sh "x:g9" componentc r03_component_g9 > gpurun_out/r03a_pmc_comp.json && \
bash scripts/pmc_kernel.sh "x:m8" componentc r03_component_m8 > gpurun_out/r03a_pmc_m8.json && \
bash scripts/pmc_kernel.sh "x:g9deep" treec r03_tree_g9deep > gpurun_out/r03a_pmc_g9deep.json && \
bash scripts/pmc_kernel.sh "x:p8" tree_384 r03_tree_p8 > gpurun_out/r03a_pmc_p8.json
rc=$?; cut -c1-600 gpurun_out/r03a_pmc_*.json; exit $rc
