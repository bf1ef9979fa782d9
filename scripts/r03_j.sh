#!/bin/bash
# round 3: what bounds the component and tree kernels at HEAD (stores, invariants, level counts)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u scripts/probe.py "g9:g9" "g9nostore:g9||TLCG_NO_STORE" "g9noinv:g9||TLCG_NO_INV" "g9nolvl:g9||TLCG_NO_LVL" "g9none:g9||TLCG_NO_STORE;TLCG_NO_INV;TLCG_NO_LVL" "m8:m8" "m8nostore:m8||TLCG_NO_STORE" "g9deep:g9deep" "g9deepnostore:g9deep||TLCG_TREE_NO_STORE" "g9deepnoinv:g9deep||TLCG_TREE_NO_INV" "g9:g9" > gpurun_out/r03j_probe.jsonl 2>&1; rc=$?; cut -c1-220 gpurun_out/r03j_probe.jsonl; exit $rc
