#!/bin/bash
# SQ counters of the component-tree kernel on P8 (one group per rocprofv3 pass)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/sqt
cat > /tmp/one_tree.py <<'PY'
import os, sys
sys.path.insert(0, os.path.join(os.environ["GRAFT_REPO_ROOT"], "pulsar-tlaplus_amd", "python"))
import tlcgpu as T
m = T.Model(key_space=range(1, 8), value_space=range(1, 8), model_producer=True, retain_null_key=False)
ck = T.Checker(m, engine="tree")
st = ck.run_raw(); print(st.generated, st.distinct, st.kernel_ms, st.engine)
PY
i=0
for ctr in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/sqt/p$i -o run -- python -u /tmp/one_tree.py > gpurun_out/sqt/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/sqt/p$i.log; }
done
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sqt/kt -o run -- python -u /tmp/one_tree.py > gpurun_out/sqt/kt.log 2>&1 || echo "kernel trace failed"
python3 - <<'PY'
import csv, glob, collections
for d in sorted(glob.glob("gpurun_out/sqt/p*/run_counter_collection.csv")):
    agg = collections.defaultdict(float)
    for r in csv.DictReader(open(d)):
        if "k_tree" in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
    for k, v in agg.items(): print(k, "%.4g" % v)
for r in csv.DictReader(open("gpurun_out/sqt/kt/run_kernel_trace.csv")):
    if "k_tree" in r["Kernel_Name"]:
        print("launch", (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6, "ms")
PY
