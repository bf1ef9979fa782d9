#!/bin/bash
# round 3: tree closed mode with paired FPSet probes -- parity, A/B; PMC of the component kernel with store records
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_tree.py tests/test_gpu_limits.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r03l_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r03l_pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python -u scripts/probe.py "p2:g9deep" "p1:g9deep||TLCG_TREE_PROBE2=0" "p2:g9deep" "p1:g9deep||TLCG_TREE_PROBE2=0" > gpurun_out/r03l_probe.jsonl 2>&1; rc=$?; cut -c1-200 gpurun_out/r03l_probe.jsonl; [ $rc = 0 ] || exit $rc
bash scripts/pmc_kernel.sh "x:g9" componentc r03_component_g9 > gpurun_out/r03l_pmc_component_g9.json && \
bash scripts/pmc_kernel.sh "x:m8" componentc r03_component_m8 > gpurun_out/r03l_pmc_component_m8.json && \
bash scripts/pmc_kernel.sh "x:g9deep" treec r03_tree_g9deep > gpurun_out/r03l_pmc_tree_g9deep.json; rc=$?; cut -c1-300 gpurun_out/r03l_pmc_*.json; exit $rc
