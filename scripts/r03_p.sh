#!/bin/bash
# round 3: component kernel with the successors' invariants evaluated before their probes (A/B)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u scripts/probe.py "base:g9" "spec:g9||TLCG_SPEC_INV=1" "base:g9" "spec:g9||TLCG_SPEC_INV=1" "base:m8" "spec:m8||TLCG_SPEC_INV=1" > gpurun_out/r03p_probe.jsonl 2>&1; rc=$?; cut -c1-200 gpurun_out/r03p_probe.jsonl; exit $rc
