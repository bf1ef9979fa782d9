#!/bin/bash
# round 3: Producer mode's invariants at expansion vs at insert (P8); every GPU test first
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r03an_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r03an_pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python -u scripts/probe.py "expand:p8" "insert:p8||TLCG_TREE_INV_AT_EXPAND_OPEN=0" "expand:p8" "insert:p8||TLCG_TREE_INV_AT_EXPAND_OPEN=0" "expand:p8" "insert:p8||TLCG_TREE_INV_AT_EXPAND_OPEN=0" > gpurun_out/r03an_probe.jsonl 2>&1; rc=$?; cut -c1-200 gpurun_out/r03an_probe.jsonl; exit $rc
