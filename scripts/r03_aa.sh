#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 150 --timeout-method thread -k "records_decode" > gpurun_out/r03aa_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r03aa_pytest.log; exit $rc
