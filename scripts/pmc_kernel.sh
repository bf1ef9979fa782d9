#!/bin/bash
# PMC counters (SQ issue/LDS groups, FETCH_SIZE, WRITE_SIZE: one group per
# rocprofv3 pass) and a kernel trace of one complete check, for the kernels
# whose name contains $2.
#   scripts/pmc_kernel.sh CASE KERNEL_SUBSTRING OUTNAME
# CASE is a scripts/probe.py case (e.g. "x:g9deep", "x:g9:0/8|TLCG_COMP_GRID=3072").
# Writes gpurun_out/pmc/OUTNAME/ and prints a JSON summary (scripts/pmc_summarize.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; export PROBE_REPS=1
CASE="$1"; KSUB="$2"; OUT="gpurun_out/pmc/$3"
mkdir -p "$OUT"
# CASE "node:W,KEYS,CHECKS": scripts/node_bench.py W KEYS CHECKS instead of a probe case
if [ "${CASE#node:}" != "$CASE" ]; then
  IFS=',' read -r -a RUN <<< "${CASE#node:}"; RUN=(scripts/node_bench.py "${RUN[@]}")
else
  RUN=(scripts/probe.py "$CASE")
fi
i=0
for ctr in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $ctr --output-format csv -d "$OUT/p$i" -o run -- python3 -u "${RUN[@]}" > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
done
timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o run -- python3 -u "${RUN[@]}" > "$OUT/kt.log" 2>&1 || { echo "kernel trace failed"; exit 1; }
python3 scripts/pmc_summarize.py "$OUT" "$KSUB" "$CASE"
