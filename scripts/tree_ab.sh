set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_tree.py tests/test_gpu_parity.py -k "tree or p8 or P_ or producer" -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tree.log 2>&1; tail -5 gpurun_out/tree.log
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --config p8 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/p8_tree_$i.json 2>gpurun_out/p8_tree_$i.err || { tail gpurun_out/p8_tree_$i.err; exit 1; }
  TLCG_TREE=0 timeout -k 10 300 python -u bench.py --config p8 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/p8_glob_$i.json 2>/dev/null || exit 1
done
for f in gpurun_out/p8_tree_*.json gpurun_out/p8_glob_*.json; do python3 -c "import json,sys; d=json.load(open('$f')); print('$f', d['ms_per_step'], d['config'].get('gpu_kernel_ms_per_step'), d['config'].get('engine'), d['value'])"; done
