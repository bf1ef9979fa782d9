cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
for v in "TLCG_JIT=1" "TLCG_JIT_DEFINES=TLCG_TREE_KEYS_HBM" "TLCG_JIT_DEFINES=TLCG_TREE_KEYS_HBM;TLCG_TREE_TSCALE=105" "TLCG_JIT_DEFINES=TLCG_TREE_KEYS_HBM;TLCG_TREE_TSCALE=120" "TLCG_JIT_DEFINES=TLCG_TREE_TSCALE=105" "TLCG_JIT=1"; do
  env "$v" timeout -k 10 300 python -u bench.py --config p8 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/p8_ab.json 2>gpurun_out/p8_ab.err || { tail -5 gpurun_out/p8_ab.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/p8_ab.json')); print('$v', d['ms_per_step'], d['config'].get('gpu_kernel_ms_per_step'), d['config'].get('engine'), '%.4g' % d['value'])"
done
