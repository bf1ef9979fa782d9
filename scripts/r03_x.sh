#!/bin/bash
# round 3: the component code pass's records in their own buffer (the store holds only the cascade): parity
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_partition.py tests/test_gpu_random_cfgs.py tests/test_gpu_cli.py tests/test_gpu_dist.py tests/test_gpu_liveness.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r03x_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r03x_pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python -u scripts/probe.py "g9:g9" "m8:m8" "sh:g9:0/8" > gpurun_out/r03x_probe.jsonl 2>&1; rc=$?; cut -c1-200 gpurun_out/r03x_probe.jsonl; exit $rc
