"""Summarize scripts/pmc_sq.sh output (one counter group per rocprofv3 pass)
into profiles/<round>_pmc_component.json for the component kernel."""
import collections, csv, glob, json, os, sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/sq"
out = sys.argv[2] if len(sys.argv) > 2 else "profiles/r02_pmc_component.json"
DISTINCT = 1_040_187_392  # G9
agg, kname = collections.defaultdict(float), None
for f in sorted(glob.glob(os.path.join(root, "p*", "run_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        if "component" in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            kname = r["Kernel_Name"]
c = dict(agg)
hbm = (c.get("FETCH_SIZE", 0) + c.get("WRITE_SIZE", 0)) * 1024  # KB -> B
summary = {
    "kernel": f"{kname} (hipRTC-specialized, G9 cfg, one full check)",
    "counters": c,
    "hbm_bytes_per_step": hbm,
    # SQ_INSTS_* count wave instructions; a wave expands 64 states (one per lane) per BFS iteration
    "valu_wave_insts_per_iteration": c.get("SQ_INSTS_VALU", 0) * 64 / DISTINCT,
    "salu_wave_insts_per_iteration": c.get("SQ_INSTS_SALU", 0) * 64 / DISTINCT,
    "lds_wave_insts_per_iteration": c.get("SQ_INSTS_LDS", 0) * 64 / DISTINCT,
    "wave_issue_frac": c.get("SQ_ACTIVE_INST_ANY", 0) / max(c.get("SQ_WAVE_CYCLES", 1), 1),
    "note": "one counter group per rocprofv3 pass (scripts/pmc_sq.sh); FETCH/WRITE_SIZE in KB; "
            "WRITE_SIZE = the 16 B/state store + parent log; SQ_*_CYCLES in quad-cycles",
}
json.dump(summary, open(out, "w"), indent=1)
print(json.dumps(summary, indent=1))
