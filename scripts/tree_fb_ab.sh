#!/bin/bash
# A/B of the component tree's LDS frontier buffer (TLCG_TREE_FB / _OPEN) on
# G9-deep (closed mode) and P8 (Producer); bench.py checks the counts
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
ab() {  # config steps variants...
  local cfg=$1 steps=$2; shift 2
  for v in "$@"; do
    TLCG_JIT_DEFINES="$v" timeout -k 10 300 python -u bench.py --config $cfg --steps $steps --warmup 1 --no-cpu-baseline > gpurun_out/fb_ab.json 2>gpurun_out/fb_ab.err || { tail -5 gpurun_out/fb_ab.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/fb_ab.json')); print(json.dumps(dict(config='$cfg', defines='$v', ms=d['ms_per_step'], kernel_ms=d['config'].get('gpu_kernel_ms_per_step'), engine=d['config'].get('engine'), value=d['value'])))" | tee -a gpurun_out/fb_ab.jsonl
  done
}
ab ${CFG1:-g9deep} 3 ${V1:-"" "TLCG_TREE_FB=32" "TLCG_TREE_FB=16" ""}
ab ${CFG2:-p8} 5 ${V2:-"" "TLCG_TREE_FB_OPEN=32" "TLCG_TREE_FB_OPEN=16" ""}
