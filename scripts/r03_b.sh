#!/bin/bash
# round 3: what costs M8 / the 1/8 share per state (grid, per-level atomics), tree group sizes
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u scripts/probe.py \
  "m8:m8" "m8nolvl:m8||TLCG_NO_LVL" "m8g4096:m8|TLCG_COMP_GRID=4096" "m8g6144:m8|TLCG_COMP_GRID=6144" "m8g8192:m8|TLCG_COMP_GRID=8192" "m8g12288:m8|TLCG_COMP_GRID=12288" "m8g6144nolvl:m8|TLCG_COMP_GRID=6144|TLCG_NO_LVL" \
  "sh0:g9:0/8" "sh0nolvl:g9:0/8||TLCG_NO_LVL" "sh0g6144:g9:0/8|TLCG_COMP_GRID=6144" "sh0g8192:g9:0/8|TLCG_COMP_GRID=8192" \
  "g9:g9" "g9nolvl:g9||TLCG_NO_LVL" "g9g32768:g9|TLCG_COMP_GRID=32768" "g9g131072:g9|TLCG_COMP_GRID=131072" "g9g262144:g9|TLCG_COMP_GRID=262144" \
  "g9deep:g9deep" "g9deepG8:g9deep||TLCG_TREEC_G=8" "g9deepG2:g9deep||TLCG_TREEC_G=2" "g9deep:g9deep" \
  > gpurun_out/r03b_probe.jsonl 2>&1; rc=$?; cut -c1-260 gpurun_out/r03b_probe.jsonl; exit $rc
