#!/bin/bash
# component-tree engine: its GPU tests, then P8 with 1 / 2 / 4 components per
# wavefront (TLCG_TREE_G) and the global engine (TLCG_TREE=0), twice each
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_tree.py tests/test_gpu_parity.py -k "tree or p8 or P_ or producer" -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tree.log 2>&1; tail -5 gpurun_out/tree.log
for i in 1 2; do
  for v in ${VARIANTS:-"TLCG_JIT=1" "TLCG_JIT=0" "TLCG_TREE=0"}; do
    env $v timeout -k 10 300 python -u bench.py --config ${CFG:-p8} --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/tree_ab.json 2>gpurun_out/tree_ab.err || { tail -5 gpurun_out/tree_ab.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/tree_ab.json')); print('$v', d['ms_per_step'], d['config'].get('gpu_kernel_ms_per_step'), d['config'].get('engine'), '%.4g' % d['value'])"
  done
done
