#!/bin/bash
# round 3: tree closed mode, a candidate's invariants evaluated while its first CAS is in flight (A/B + parity)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TLCG_JIT_DEFINES="TLCG_TREE_SPEC_INV=1" timeout -k 10 600 python -u -m pytest tests/test_gpu_tree.py tests/test_gpu_parity.py -m gpu -x -q --timeout 150 --timeout-method thread -k "tree or g9deep or wide or W_" > gpurun_out/r03s_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r03s_pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python -u scripts/probe.py "base:g9deep" "spec:g9deep||TLCG_TREE_SPEC_INV=1" "base:g9deep" "spec:g9deep||TLCG_TREE_SPEC_INV=1" > gpurun_out/r03s_probe.jsonl 2>&1; rc=$?; cut -c1-200 gpurun_out/r03s_probe.jsonl; exit $rc
