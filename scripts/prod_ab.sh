#!/bin/bash
# Producer-mode global engine: the fast kernel vs the general one (TLCG_FAST_ITEMS=0), P8 bench, then the
# producer-mode parity tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --config p8 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/p8_fast_$i.json 2>/dev/null || exit 1
  TLCG_FAST_ITEMS=0 timeout -k 10 300 python -u bench.py --config p8 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/p8_gen_$i.json 2>/dev/null || exit 1
done
for f in gpurun_out/p8_*.json; do python3 -c "import json,sys; d=json.load(open('$f')); print('$f', d['ms_per_step'], d['config']['gpu_kernel_ms_per_step'], d['value'])"; done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_random_cfgs.py tests/test_gpu_spill.py tests/test_gpu_fpset_tier.py tests/test_gpu_partition.py tests/test_gpu_checkpoint.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pt.log 2>&1; tail -4 gpurun_out/pt.log
