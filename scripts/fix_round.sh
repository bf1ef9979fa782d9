#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_cli.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/fix.log 2>&1; tail -15 gpurun_out/fix.log
timeout -k 10 400 python -u scripts/comp_variants.py "" "TLCG_HWIT_OFF" "" "TLCG_HWIT_OFF" > gpurun_out/cv.log 2>&1; cat gpurun_out/cv.log
