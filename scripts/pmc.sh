#!/bin/bash
# HBM traffic of k_expand (one G9 step) + calibration on the scattered-access
# microbenchmark; one counter group per rocprofv3 pass (MI355X_MICROARCH.md).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
timeout -s KILL 60 rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1 || true
for ctr in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" "TCC_EA0_ATOMIC_sum"; do
  tag=$(echo $ctr | tr ' ' '_')
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/pmc/bench_$tag -o run -- python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmc/bench_$tag.log 2>&1 || { echo "bench pass $ctr failed"; tail -5 gpurun_out/pmc/bench_$tag.log; }
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/pmc/micro_$tag -o run -- ./pulsar-tlaplus_amd/bin/fpset_microbench 31 268435456 > gpurun_out/pmc/micro_$tag.log 2>&1 || { echo "micro pass $ctr failed"; tail -5 gpurun_out/pmc/micro_$tag.log; }
done
ls gpurun_out/pmc
