"""Docs helper (CPU): rewrite BASELINE.md's measured-results table from the
newest round's bench lines, profiles/rNN_bench_<cfg>.json (one JSON line
each, as bench.py prints it).

    python scripts/baseline_table.py [rNN]
"""
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
rnd = sys.argv[1] if len(sys.argv) > 1 else sorted(
    os.path.basename(p)[:3] for p in glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]_bench_g9.json")))[-1]
b = {c: json.load(open(os.path.join(ROOT, "profiles", f"{rnd}_bench_{c}.json")))
     for c in ["g9", "m8", "p8", "g9deep", "g9u", "g9uall"]}


def f3(x):
    return f"{x:.3g}"


def ms(x):
    return f"{x:.3f}".rstrip("0").rstrip(".") if x < 10 else f"{x:.2f}"


def frac(r):
    return f"{r['frac']:.2f}" if r["frac"] >= 0.1 else f"{r['frac']:.3f}"


def traffic(r):
    t = r.get("traffic")
    if t is None:
        return "--"
    gb = r.get("traffic_bytes_per_step", 0) / 1e9
    return f"{t:,.0f} GB/s = {gb:.2f} GB per check ({t / r['peak']:.2f} of peak)"


rows = ["| config | G | engine (kernel) | distinct/s | BFS wall (ms) | SURVEY 8(d) frac | HBM traffic (PMC) | expansions / distinct | port distinct/s (cores) |",
        "|---|---|---|---|---|---|---|---|---|"]


def head(name, d, label, notional):
    r = d["roofline"]
    cb = d.get("cpu_baseline") or {}
    port = f"{f3(cb['value'])} ({cb['cores']})" if cb.get("value") else ""
    fr = frac(r) + (" (notional: through LDS)" if notional else "")
    rows.append(f"| {name} | 1 | {label} | **{f3(d['value'])}** | **{ms(d['ms_per_step'])}** (kernel {ms(r['avg_launch_ms'] * r.get('launches_per_step', 1))}) "
                f"| {fr} | {traffic(r)} | {d.get('distinct_per_expansion', '--')} | {port} |")


def glob_row(name, d):
    g = d["engines"]["global_hbm_fpset"]
    gr = g["roofline"]
    extra = ""
    if gr.get("traffic_over_algorithmic"):
        sa = gr.get("scattered_access_roofline", {})
        extra = f" ({gr['traffic_over_algorithmic']}x the algorithmic bytes; {sa.get('frac')} of the scattered-access roofline)"
    t = f"{gr['traffic']:,.0f} GB/s{extra}" if gr.get("traffic") else "--"
    rows.append(f"| {name} | 1 | global, HBM FPSet (`k_expand_fast`, layout-specialized where it applies) | {f3(g['value'])} | {ms(g['ms_per_step'])} | {frac(gr)} | {t} | {g.get('distinct_per_expansion', '--')} | |")


def wave_row(name, d, label):
    w = d["engines"].get("wave_quotient")
    if w:
        rows.append(f"| {name} | 1 | *quotient:* {label} | ({f3(w['value_quotient'])}, not per-state) | {ms(w['ms_per_step'])} | -- | -- | {w['states_per_expansion']:.0f} | |")


head("G9 (1.04G)", b["g9"], "component, per lane, bitmap FPSet, table-driven compactor step (`tlcg_componentp_64`, round 6)", True)
rows.append("| G9 | 1 | component, per lane (`tlcg_componentc_64`, rounds 2-5) | 2.2e11 | 4.67-4.72 | 0.96 | 870 GB/s | 1.0 | |")
glob_row("G9", b["g9"])
wave_row("G9", b["g9"], "one code-graph walk per wavefront for 16 x 64 components (`tlcg_componentw_64`, round 5)")
head("M8 (109.8M)", b["m8"], "component, per lane (`tlcg_componentp_64`)", True)
glob_row("M8", b["m8"])
wave_row("M8", b["m8"], "10 x 64 components per walk")
head("P8 (91.8M, Producer)", b["p8"], "component tree, 4 components per wavefront, double-hashed LDS tables, 48-key frontier buffers (`tlcg_tree_384`, round 6)", True)
rows.append("| P8 | 1 | the same before round 6 (linear probing, keys read back from HBM) | 5.0e10 | 1.83 | 0.22 | -- | -- | |")
glob_row("P8", b["p8"])
rows.append("| P8 | 8 ranks on one GPU | component tree split by subtrees | 0.90-1.19 ms of kernel per rank (`profiles/r03_p8_tree_sharded_ranks.jsonl`) | | | | | |")
head("G9-deep (986.8M, 93-bit)", b["g9deep"], "component tree, closed mode, bitmap FPSet, 16 components per wavefront (`tlcg_treecb_640`, round 6)", True)
rows.append("| G9-deep | 1 | the same with code tables, 4 per wavefront (`tlcg_treec_640`, rounds 2-5) | 5.9e10 | 16.6 | 0.26 | -- | -- | |")
glob_row("G9-deep", b["g9deep"])
wave_row("G9-deep", b["g9deep"], "`tlcg_treecw_640`, 10 x 64 components per walk")
head("G9 + `LatestIsLast` (config 5)", b["g9u"], "component, per lane (`tlcg_componentp_64`)", True)
glob_row("G9 + `LatestIsLast`", b["g9u"])
head("G9 + six user invariants", b["g9uall"], "component, per lane (`tlcg_componentp_64`)", True)
wave_row("G9 + six user invariants", b["g9uall"], "4 x 64 components per walk")
rows.append("| G9 partition 2 (config 4, round 6 at HEAD, `profiles/r06_node_final.jsonl`) | 8 ranks on one GPU | global, exchange (pull, one wait per level) | 7.7e9 | 133-136 (1.30x one context, 104 on the same box; earlier this round on another box 141-142 against 87) | -- | -- | -- | -- |")
rows.append("| G9 partition 2 (config 4, round 6 at HEAD) | 2 ranks on one GPU | the same | 1.05e10 | 99 (0.95x one context) | -- | -- | -- | -- |")

p = os.path.join(ROOT, "BASELINE.md")
s = open(p).read()
start = s.index("| config | G | engine (kernel) | distinct/s |")
end = s.index("Errors reported as TLC reports them")
s = s[:start] + "\n".join(rows) + "\n\n" + s[end:]
open(p, "w").write(s)
print(f"{rnd}: {len(rows) - 2} rows")
