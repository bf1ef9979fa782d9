#!/bin/bash
# The one evidence script for GPU-box runs (gpurun): each step under its own
# time limit, the steps chained so the first failure ends the call.
#
#   scripts/gpu.sh STEP [STEP ...]
#
# STEP (arguments after ':' are split on ','):
#   smoke                         __graft_entry__.smoke()
#   tests:ARGS                    pytest -m gpu ARGS (e.g. tests:tests/test_gpu_user_inv.py)
#   bench:NAME:ARGS               bench.py ARGS  -> gpurun_out/bench_NAME.json (the JSON line)
#   prof:NAME:ARGS                rocprofv3 --kernel-trace --stats of bench.py ARGS -> gpurun_out/prof_NAME/
#   pmc:NAME:KERNEL:CASE          PMC groups of one check (scripts/pmc_kernel.sh CASE KERNEL NAME)
#   probe:NAME:CASE,CASE,...      scripts/probe.py CASEs -> gpurun_out/probe_NAME.jsonl
#   node:NAME:ARGS                scripts/node_bench.py ARGS -> gpurun_out/node_NAME.jsonl
#   nodeprof:NAME:ARGS            rocprofv3 --kernel-trace of node_bench ARGS -> gpurun_out/timeline_NAME.jsonl
#   py:NAME:SCRIPT,ARGS           python SCRIPT ARGS -> gpurun_out/py_NAME.log
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for step in "$@"; do
  kind="${step%%:*}"
  rest="${step#*:}"
  [ "$rest" = "$step" ] && rest=""
  echo "== $step"
  case "$kind" in
    smoke)
      timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
        || { echo "smoke failed"; tail -30 gpurun_out/smoke.log; exit 1; }
      tail -1 gpurun_out/smoke.log ;;
    tests)
      IFS=',' read -r -a args <<< "$rest"
      timeout -k 10 1100 python -u -m pytest -m gpu --maxfail=10 -v --timeout 120 --timeout-method thread "${args[@]}" \
        > gpurun_out/gputest.log 2>&1
      rc=$?
      tail -25 gpurun_out/gputest.log
      [ $rc -eq 0 ] || { echo "gpu tests rc=$rc"; exit 1; } ;;
    bench)
      name="${rest%%:*}"; a="${rest#*:}"; [ "$a" = "$rest" ] && a=""
      IFS=',' read -r -a args <<< "$a"
      timeout -k 10 400 python -u bench.py "${args[@]}" > "gpurun_out/bench_$name.log" 2>&1 \
        || { echo "bench $name failed"; tail -20 "gpurun_out/bench_$name.log"; exit 1; }
      tail -1 "gpurun_out/bench_$name.log" > "gpurun_out/bench_$name.json"
      cut -c1-600 "gpurun_out/bench_$name.json" ;;
    prof)
      name="${rest%%:*}"; a="${rest#*:}"; [ "$a" = "$rest" ] && a=""
      IFS=',' read -r -a args <<< "$a"
      timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "gpurun_out/prof_$name" -o run \
        -- python3 -u bench.py "${args[@]}" > "gpurun_out/prof_$name.log" 2>&1 \
        || { echo "prof $name failed"; tail -20 "gpurun_out/prof_$name.log"; exit 1; }
      f=$(ls gpurun_out/prof_$name/*/run_kernel_stats.csv gpurun_out/prof_$name/run_kernel_stats.csv 2>/dev/null | head -1)
      [ -n "$f" ] && head -6 "$f" | cut -c1-200 ;;
    pmc)
      IFS=':' read -r name ksub case <<< "$rest"
      timeout -k 10 900 bash scripts/pmc_kernel.sh "$case" "$ksub" "$name" > "gpurun_out/pmc_$name.log" 2>&1 \
        || { echo "pmc $name failed"; tail -20 "gpurun_out/pmc_$name.log"; exit 1; }
      tail -3 "gpurun_out/pmc_$name.log" | cut -c1-800 ;;
    probe)
      name="${rest%%:*}"; a="${rest#*:}"
      IFS=',' read -r -a args <<< "$a"
      timeout -k 10 900 python -u scripts/probe.py "${args[@]}" > "gpurun_out/probe_$name.jsonl" 2>&1 \
        || { echo "probe $name failed"; tail -20 "gpurun_out/probe_$name.jsonl"; exit 1; }
      cut -c1-300 "gpurun_out/probe_$name.jsonl" ;;
    node)
      name="${rest%%:*}"; a="${rest#*:}"; [ "$a" = "$rest" ] && a=""
      IFS=',' read -r -a args <<< "$a"
      timeout -k 10 600 python -u scripts/node_bench.py "${args[@]}" > "gpurun_out/node_$name.jsonl" 2>&1 \
        || { echo "node $name failed"; tail -20 "gpurun_out/node_$name.jsonl"; exit 1; }
      cut -c1-400 "gpurun_out/node_$name.jsonl" ;;
    nodeprof)
      name="${rest%%:*}"; a="${rest#*:}"; [ "$a" = "$rest" ] && a=""
      IFS=',' read -r -a args <<< "$a"
      timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d "gpurun_out/nodeprof_$name" -o run \
        -- python3 -u scripts/node_bench.py "${args[@]}" > "gpurun_out/nodeprof_$name.log" 2>&1 \
        || { echo "nodeprof $name failed"; tail -20 "gpurun_out/nodeprof_$name.log"; exit 1; }
      f=$(ls gpurun_out/nodeprof_$name/*/run_kernel_trace.csv gpurun_out/nodeprof_$name/run_kernel_trace.csv 2>/dev/null | head -1)
      [ -n "$f" ] && python3 scripts/timeline.py "$f" > "gpurun_out/timeline_$name.jsonl" && cut -c1-600 "gpurun_out/timeline_$name.jsonl"
      ;;
    py)
      name="${rest%%:*}"; a="${rest#*:}"
      IFS=',' read -r -a args <<< "$a"
      timeout -k 10 600 python -u "${args[@]}" > "gpurun_out/py_$name.log" 2>&1 \
        || { echo "py $name failed"; tail -20 "gpurun_out/py_$name.log"; exit 1; }
      cut -c1-400 "gpurun_out/py_$name.log" | tail -20 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "ALL DONE"
