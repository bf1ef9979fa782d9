#!/bin/bash
# G9-deep: the component tree's closed mode vs the wide global engine, and the
# parity tests of the closed mode (wide golden cases, G9-deep counts)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "W_ or R_ or g9deep or X_ or golden_case" -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/deep.log 2>&1; tail -5 gpurun_out/deep.log
for v in ${VARIANTS:-"TLCG_JIT=1" "TLCG_JIT=0" "TLCG_TREE=0"}; do
  env $v timeout -k 10 300 python -u bench.py --config g9deep --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/deep_ab.json 2>gpurun_out/deep_ab.err || { tail -5 gpurun_out/deep_ab.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/deep_ab.json')); print('$v', d['ms_per_step'], d['config'].get('gpu_kernel_ms_per_step'), d['config'].get('engine'), '%.4g' % d['value'])"
done
