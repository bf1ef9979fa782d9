#!/bin/bash
# A/B of component-kernel variants given as arguments (hipRTC define sets),
# each twice, interleaved, on one box; then the component-engine parity tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u scripts/comp_variants.py "$@" "$@" > gpurun_out/cv.log 2>&1; cat gpurun_out/cv.log
[ -n "$NOTEST" ] || timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_random_cfgs.py tests/test_gpu_limits.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pt.log 2>&1; tail -5 gpurun_out/pt.log
