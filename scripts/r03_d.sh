#!/bin/bash
# round 3: the component tree's closed mode (G9-deep) -- table size, slot hash, what the stores / invariants cost
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u scripts/probe.py \
  "base:g9deep" "t1024:g9deep||TLCG_TREE_TSCALE_CLOSED=160" "t768:g9deep||TLCG_TREE_TSCALE_CLOSED=120" \
  "mult:g9deep||TLCG_TREE_MULT=0x932d0489u" "nostore:g9deep||TLCG_TREE_NO_STORE" "noinv:g9deep||TLCG_TREE_NO_INV" \
  "t1024g2:g9deep|TLCG_TREE_G=2|TLCG_TREE_TSCALE_CLOSED=160;TLCG_TREEC_G=2" "base:g9deep" \
  > gpurun_out/r03d_probe.jsonl 2>&1; rc=$?; cut -c1-200 gpurun_out/r03d_probe.jsonl; exit $rc
