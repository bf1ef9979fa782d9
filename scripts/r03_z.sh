#!/bin/bash
# round 3: tree closed mode at 8 components per wavefront (8-lane groups) against 4, at HEAD
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u scripts/probe.py "g4:g9deep" "g8:g9deep||TLCG_TREEC_G=8" "g4:g9deep" "g8:g9deep||TLCG_TREEC_G=8" > gpurun_out/r03z_probe.jsonl 2>&1; rc=$?; cut -c1-200 gpurun_out/r03z_probe.jsonl; exit $rc
