#!/bin/bash
# one GPU verification round: smoke, -m gpu tests, bench, rocprofv3 kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; tail -30 gpurun_out/smoke.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=10 -v --timeout 120 --timeout-method thread ${GPU_TEST_ARGS:-} > gpurun_out/gputest.log 2>&1
rc=$?
tail -40 gpurun_out/gputest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "gpu tests aborted rc=$rc"; exit 1; }
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1 || { echo bench failed; tail -20 gpurun_out/bench.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof.log 2>&1 || { echo prof failed; tail -20 gpurun_out/prof.log; exit 1; }
echo "ALL DONE tests rc=$rc"
tail -3 gpurun_out/smoke.log; cat gpurun_out/bench.log
