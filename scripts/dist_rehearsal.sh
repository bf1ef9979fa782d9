#!/bin/bash
# 2 ranks on one GPU over gloo: exercises bench.py's multi-rank path (the driver runs N=2..8 with RCCL)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --dist-backend gloo > gpurun_out/bench_n2_gloo.log 2>&1; echo rc=$?
tail -3 gpurun_out/bench_n2_gloo.log
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > gpurun_out/bench_n1.log 2>&1; echo rc=$?
tail -2 gpurun_out/bench_n1.log
