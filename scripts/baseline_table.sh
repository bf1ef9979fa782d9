#!/bin/bash
# one bench line per config (BASELINE.md "Measured results"); the port CPU
# baseline once, on G9
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
: > gpurun_out/baseline.jsonl
for c in s m8 p8 g9deep; do
  timeout -k 10 300 python -u bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline >> gpurun_out/baseline.jsonl 2>gpurun_out/baseline_$c.err || { echo "bench $c failed"; tail -5 gpurun_out/baseline_$c.err; exit 1; }
done
timeout -k 10 300 python -u bench.py --config g9 --steps 10 --warmup 3 >> gpurun_out/baseline.jsonl 2>gpurun_out/baseline_g9.err || { echo "bench g9 failed"; exit 1; }
wc -l gpurun_out/baseline.jsonl
