#!/bin/bash
# round 3 final evidence at HEAD: every GPU test, smoke, PMC of the tree kernels (pair mode),
# benches (G9 under rocprofv3 --stats, G9, M8, P8, G9-deep), G9 at 8 virtual ranks
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > gpurun_out/r03ao_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r03ao_pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03ao_smoke.log 2>&1 || exit 1
cat gpurun_out/r03ao_smoke.log
bash scripts/pmc_kernel.sh "x:g9deep" treec r03_tree_g9deep > gpurun_out/r03ao_pmc_tree_g9deep.json && \
bash scripts/pmc_kernel.sh "x:p8" tree_384 r03_tree_p8 > gpurun_out/r03ao_pmc_tree_p8.json || exit 1
cp gpurun_out/r03ao_pmc_tree_g9deep.json profiles/r03_pmc_tree_g9deep.json && cp gpurun_out/r03ao_pmc_tree_p8.json profiles/r03_pmc_tree_p8.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03ao_bench_g9 -o run -- python3 -u bench.py --steps 10 --warmup 3 > gpurun_out/r03ao_bench_g9.json 2> gpurun_out/r03ao_bench_g9.err || exit 1
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 > gpurun_out/r03ao_bench_g9_plain.json 2> gpurun_out/r03ao_bench_g9_plain.err || exit 1
for cfg in m8 p8 g9deep; do
  timeout -k 10 300 python3 -u bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r03ao_bench_$cfg.json 2> gpurun_out/r03ao_bench_$cfg.err || exit 1
  echo "$cfg done"
done
TLCG_RANK_TRACE=1 timeout -k 10 300 python -u scripts/node_bench.py 8 15 > gpurun_out/r03ao_node8_g9.jsonl 2> gpurun_out/r03ao_node8_g9.trace || exit 1
echo all done
