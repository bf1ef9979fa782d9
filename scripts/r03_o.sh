#!/bin/bash
# round 3: the counterexample walked across the ranks' stores -- partition, dist, CLI and parity GPU tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_partition.py tests/test_gpu_dist.py tests/test_gpu_cli.py tests/test_gpu_parity.py -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/r03o_pytest.log 2>&1; rc=$?; tail -5 gpurun_out/r03o_pytest.log; grep -c PASSED gpurun_out/r03o_pytest.log; exit $rc
