#!/bin/bash
# round 3: user invariants on the GPU (engine tests, CLI), then the tree variants
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_user_inv.py tests/test_gpu_cli.py -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/r03e_pytest.log 2>&1; rc=$?; tail -5 gpurun_out/r03e_pytest.log; [ $rc = 0 ] || exit $rc
bash scripts/r03_d.sh
