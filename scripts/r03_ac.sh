#!/bin/bash
# round 3: what 8 components per wavefront would give at equal occupancy -- 4 per wavefront padded to 8 workgroups per CU
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u scripts/probe.py "g4:g9deep" "g4pad8:g9deep||TLCG_TREE_LDS_PAD=7680" "g8:g9deep||TLCG_TREEC_G=8" "g4pad8:g9deep||TLCG_TREE_LDS_PAD=7680" > gpurun_out/r03ac_probe.jsonl 2>&1; rc=$?; cut -c1-200 gpurun_out/r03ac_probe.jsonl; exit $rc
