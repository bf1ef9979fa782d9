"""Summarize scripts/pmc_kernel.sh output: the counters of the kernels whose
name contains KSUB, summed over their dispatches, per-launch averages from the
kernel trace, the issue fraction and the HBM bytes.

    python scripts/pmc_summarize.py DIR KSUB CASE [OUT.json]

HBM bytes (MI355X_MICROARCH.md, HBM): FETCH_SIZE and WRITE_SIZE are in KB;
on gfx950 FETCH_SIZE tallies 128-B read requests of wide streaming reads at
64 B, so it is doubled ("fetch_bytes_corrected"); WRITE_SIZE is taken as is.
PMC_FETCH_SCALE=1 keeps FETCH_SIZE as counted: scattered 8-B loads count one
64-B request each (profiles/r03_pmc_calibration.json), so a probe-bound
kernel (k_expand_fast) is summarized with it."""
import collections
import csv
import glob
import json
import os
import sys

root, ksub, case = sys.argv[1], sys.argv[2], sys.argv[3]
out = sys.argv[4] if len(sys.argv) > 4 else None
CUS, SIMDS, CLOCK_HZ = 256, 4, 2.4e9
agg, names = collections.defaultdict(float), set()
for f in sorted(glob.glob(os.path.join(root, "p*", "run_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        if ksub in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            names.add(r["Kernel_Name"])
durs = []
for f in glob.glob(os.path.join(root, "kt", "run_kernel_trace.csv")):
    for r in csv.DictReader(open(f)):
        if ksub in r["Kernel_Name"]:
            durs.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
c = dict(agg)
# the probe runs one check per pass (PROBE_REPS=1); the trace's launches are that check's
kt = sum(durs)
fscale = float(os.environ.get("PMC_FETCH_SCALE", "2"))
fetch = c.get("FETCH_SIZE", 0.0) * 1024 * fscale
write = c.get("WRITE_SIZE", 0.0) * 1024
res = dict(case=case, kernels=sorted(names), launches=len(durs), kernel_s=kt, counters=c,
           fetch_bytes_corrected=fetch, write_bytes=write, hbm_bytes=fetch + write,
           note=f"one counter group per rocprofv3 pass; FETCH_SIZE x 1024 x {fscale:g} (x2: gfx950 tallies 128-B "
                "streaming reads at 64 B; x1: scattered probes, one 64-B request each), WRITE_SIZE x 1024; "
                "SQ_*_CYCLES in quad-cycles; one complete check per pass")
if kt > 0 and c:
    t_valu = c.get("SQ_INSTS_VALU", 0) * 2 / (CUS * SIMDS * CLOCK_HZ)
    t_salu = c.get("SQ_INSTS_SALU", 0) / (CUS * CLOCK_HZ)
    t_lds = c.get("SQ_LDS_IDX_ACTIVE", 0) / (CUS * CLOCK_HZ)
    res["issue"] = dict(frac=max(t_valu, t_salu, t_lds) / kt, valu_ms=t_valu * 1e3, salu_ms=t_salu * 1e3,
                        lds_ms=t_lds * 1e3,
                        wave_issue_frac=c.get("SQ_ACTIVE_INST_ANY", 0) / max(c.get("SQ_WAVE_CYCLES", 1), 1),
                        wait_any_frac=c.get("SQ_WAIT_ANY", 0) / max(c.get("SQ_WAVE_CYCLES", 1), 1),
                        lds_conflict_frac=c.get("SQ_LDS_BANK_CONFLICT", 0) / max(c.get("SQ_LDS_IDX_ACTIVE", 1), 1),
                        formula="frac = max(VALU x 2 cyc / (256 CU x 4 SIMD), SALU x 1 cyc / 256 CU, "
                                "SQ_LDS_IDX_ACTIVE / 256 CU) / 2.4 GHz / kernel time")
    res["hbm_gbs"] = (fetch + write) / kt / 1e9
if out:
    json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res))
