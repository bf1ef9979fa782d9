#!/bin/bash
# one GPU verification round: smoke, -m gpu tests, bench, rocprofv3 kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; exit 1; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gputest.log 2>&1 || { echo gpu tests failed; tail -30 gpurun_out/gputest.log; exit 1; }
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1 || { echo bench failed; tail -20 gpurun_out/bench.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof.log 2>&1 || { echo prof failed; tail -20 gpurun_out/prof.log; exit 1; }
echo ALL OK
tail -3 gpurun_out/smoke.log; tail -3 gpurun_out/gputest.log; cat gpurun_out/bench.log
