#!/bin/bash
# round 3: the tree's per-depth successor sum as a DPP row scan vs ds_bpermute shuffles (G9-deep, P8)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_tree.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03ae_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r03ae_pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python -u scripts/probe.py "dpp:g9deep" "shfl:g9deep||TLCG_TREE_DPP=0" "dpp:g9deep" "shfl:g9deep||TLCG_TREE_DPP=0" "dpp:p8" "shfl:p8||TLCG_TREE_DPP=0" "dpp:p8" "shfl:p8||TLCG_TREE_DPP=0" > gpurun_out/r03ae_probe.jsonl 2>&1; rc=$?; cut -c1-220 gpurun_out/r03ae_probe.jsonl; exit $rc
