#!/bin/bash
# round 3: speculative invariants on by default -- every GPU test, smoke, G9 bench under rocprofv3, M8 bench, PMC of the component kernel
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > gpurun_out/r03q_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r03q_pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03q_smoke.log 2>&1 || exit 1
cat gpurun_out/r03q_smoke.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03q_bench_g9 -o run -- python3 -u bench.py --steps 10 --warmup 3 > gpurun_out/r03q_bench_g9.json 2> gpurun_out/r03q_bench_g9.err || exit 1
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 > gpurun_out/r03q_bench_g9_plain.json 2> gpurun_out/r03q_bench_g9_plain.err || exit 1
timeout -k 10 300 python3 -u bench.py --config m8 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r03q_bench_m8.json 2> gpurun_out/r03q_bench_m8.err || exit 1
bash scripts/pmc_kernel.sh "x:g9" componentc r03_component_g9 > gpurun_out/r03q_pmc_component_g9.json && \
bash scripts/pmc_kernel.sh "x:m8" componentc r03_component_m8 > gpurun_out/r03q_pmc_component_m8.json || exit 1
echo all done
