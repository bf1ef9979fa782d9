#!/bin/bash
# round 3: attribution of the tree's closed-mode time behind the perfect hash (experiment defines: no invariants, no stores, neither)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u scripts/probe.py "base:g9deep" "noinv:g9deep||TLCG_TREE_NO_INV" "nostore:g9deep||TLCG_TREE_NO_STORE" "neither:g9deep||TLCG_TREE_NO_INV;TLCG_TREE_NO_STORE" "base:g9deep" "noinv:g9deep||TLCG_TREE_NO_INV" "nostore:g9deep||TLCG_TREE_NO_STORE" "neither:g9deep||TLCG_TREE_NO_INV;TLCG_TREE_NO_STORE" > gpurun_out/r03al_probe.jsonl 2>&1; rc=$?; cut -c1-150 gpurun_out/r03al_probe.jsonl; exit $rc
