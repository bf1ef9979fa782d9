#!/bin/bash
# round 3: behind the perfect hash, re-check 8 components per wavefront and pair mode (G9-deep)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u scripts/probe.py "g4:g9deep" "g8:g9deep||TLCG_TREEC_G=8" "nopair:g9deep||TLCG_TREE_PAIR=0" "g4:g9deep" "g8:g9deep||TLCG_TREEC_G=8" "nopair:g9deep||TLCG_TREE_PAIR=0" > gpurun_out/r03ak_probe.jsonl 2>&1; rc=$?; cut -c1-200 gpurun_out/r03ak_probe.jsonl; exit $rc
