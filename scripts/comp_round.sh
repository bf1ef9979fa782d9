#!/bin/bash
# A/B of component-kernel variants (hipRTC defines) on one box, then the SQ
# counters of the default kernel
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/comp_variants.py "" "TLCG_SEL_STEP" "TLCG_UNIFORM_PHASE" "" "TLCG_SEL_STEP" "TLCG_UNIFORM_PHASE" > gpurun_out/cv.log 2>&1; cat gpurun_out/cv.log
[ "${PMC:-1}" = "1" ] || exit 0
timeout -k 10 600 bash scripts/pmc_sq.sh > gpurun_out/sq.log 2>&1; tail -20 gpurun_out/sq.log
