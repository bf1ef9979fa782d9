#!/bin/bash
# round 3 evidence at HEAD: every GPU test, smoke, the exchange at 8 virtual
# ranks, PMC of each engine's kernel, benches + rocprof stats
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > gpurun_out/r03h_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r03h_pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03h_smoke.log 2>&1 || exit 1
cat gpurun_out/r03h_smoke.log
TLCG_RANK_TRACE=1 timeout -k 10 300 python -u scripts/node_bench.py 8 15 > gpurun_out/r03h_node8_g9.jsonl 2> gpurun_out/r03h_node8_g9.trace || exit 1
cat gpurun_out/r03h_node8_g9.jsonl
bash scripts/pmc_kernel.sh "x:g9" componentc r03_component_g9 > gpurun_out/r03h_pmc_component_g9.json && \
bash scripts/pmc_kernel.sh "x:m8" componentc r03_component_m8 > gpurun_out/r03h_pmc_component_m8.json && \
bash scripts/pmc_kernel.sh "x:g9deep" treec r03_tree_g9deep > gpurun_out/r03h_pmc_tree_g9deep.json && \
bash scripts/pmc_kernel.sh "x:p8" tree_384 r03_tree_p8 > gpurun_out/r03h_pmc_tree_p8.json && \
PROBE_ENGINE=global bash scripts/pmc_kernel.sh "x:g9" k_expand_fast r03_expand_g9 > gpurun_out/r03h_pmc_expand_g9.json || exit 1
echo pmc done
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03h_bench_g9 -o run -- python3 -u bench.py --steps 10 --warmup 3 > gpurun_out/r03h_bench_g9.json 2> gpurun_out/r03h_bench_g9.err || exit 1
tail -c 3000 gpurun_out/r03h_bench_g9.json
for cfg in m8 p8 g9deep; do
  timeout -k 10 300 python3 -u bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r03h_bench_$cfg.json 2> gpurun_out/r03h_bench_$cfg.err || exit 1
  echo "$cfg done"
done
