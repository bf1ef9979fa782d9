#!/bin/bash
# round 3: component code pass with 32-bit store records -- parity, A/B against word stores and the DPP level sums
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r03k_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r03k_pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python -u scripts/probe.py "rec:g9" "words:g9||TLCG_COMP_CODE_STORE=0" "recu:g9||TLCG_LVL_UNIFORM=1" "rec:g9" "words:g9||TLCG_COMP_CODE_STORE=0" "recu:g9||TLCG_LVL_UNIFORM=1" "rec:m8" "recu:m8||TLCG_LVL_UNIFORM=1" "rec:g9:0/8" "recu:g9:0/8||TLCG_LVL_UNIFORM=1" > gpurun_out/r03k_probe.jsonl 2>&1; rc=$?; cut -c1-200 gpurun_out/r03k_probe.jsonl; exit $rc
