#!/bin/bash
# round 3: (1) bench.py's multi-rank path (restructured exchange leg + watchdog)
# rehearsed with 2 ranks on one GPU over gloo; (2) FETCH_SIZE / WRITE_SIZE per
# scattered 8-B access calibrated on the FPSet microbenchmark (known counts)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/cal; export TMPDIR=/tmp
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 2 --warmup 1 --config m8 --dist-backend gloo > gpurun_out/r03n_bench_n2_gloo.log 2>&1 || { echo "n2 rehearsal failed"; tail -30 gpurun_out/r03n_bench_n2_gloo.log; exit 1; }
tail -1 gpurun_out/r03n_bench_n2_gloo.log | cut -c1-400
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/cal/fetch -o run -- pulsar-tlaplus_amd/bin/fpset_microbench 31 268435456 0 > gpurun_out/cal/fetch.log 2>&1 || { echo "fetch pass failed"; tail -5 gpurun_out/cal/fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/cal/write -o run -- pulsar-tlaplus_amd/bin/fpset_microbench 31 268435456 0 > gpurun_out/cal/write.log 2>&1 || { echo "write pass failed"; tail -5 gpurun_out/cal/write.log; exit 1; }
echo cal done
