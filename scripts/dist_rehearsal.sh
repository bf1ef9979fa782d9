#!/bin/bash
# 2 ranks on one GPU over gloo: exercises bench.py's multi-rank path, including
# the open-partition all-to-all (the driver runs N=2..8 with RCCL), on M8 so the
# host-memory gloo transport stays fast
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 2 --warmup 1 --config m8 --dist-backend gloo > gpurun_out/bench_n2_gloo.log 2>&1 || { echo "n2 rehearsal failed"; tail -30 gpurun_out/bench_n2_gloo.log; exit 1; }
tail -1 gpurun_out/bench_n2_gloo.log
