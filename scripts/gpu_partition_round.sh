set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_partition.py tests/test_gpu_checkpoint.py tests/test_gpu_dist.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/gt2.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/gt2.log | tail -20
[ $rc -le 1 ] || exit 1
timeout -k 10 300 python -u scripts/node_bench.py 8 > gpurun_out/node8.log 2>&1; cat gpurun_out/node8.log | tail -4
