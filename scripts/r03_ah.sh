#!/bin/bash
# round 3: the component code pass's slots displaced by an 8-bucket perfect-hash table vs linear probing alone (G9, M8); all GPU tests first
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r03ah_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r03ah_pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python -u scripts/probe.py "disp:g9" "nodisp:g9||TLCG_COMP_DISP=0" "disp:g9" "nodisp:g9||TLCG_COMP_DISP=0" "disp:g9" "nodisp:g9||TLCG_COMP_DISP=0" "disp:m8" "nodisp:m8||TLCG_COMP_DISP=0" "disp:m8" "nodisp:m8||TLCG_COMP_DISP=0" > gpurun_out/r03ah_probe.jsonl 2>&1; rc=$?; cut -c1-200 gpurun_out/r03ah_probe.jsonl; exit $rc
