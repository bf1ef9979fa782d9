"""Kernel-time probe over configs and variants, one JSON line per run.

    python scripts/probe.py CASE [CASE ...]

CASE = name:cfg[:rank/world][|ENV=V,ENV2=V][|DEF=1;DEF2]
  cfg: s, m8, g9, g9deep, p8 (bench.py's CONFIGS)
  rank/world: a closed partition's share (e.g. 0/8: the first of 8 ranks)
  ENV: environment for the run (TLCG_COMP_GRID=3072, TLCG_TREE_G=2, ...; several
       joined by ',' or '+';
       PROBE_ENGINE=global, PROBE_TLC=1: TLC order)
  DEF: hipRTC define set (TLCG_JIT_DEFINES, e.g. TLCG_LDS_COLS=0)
Each case builds its own context, runs 3 complete checks, and reports the
best kernel time, the counts and the per-state cost (ps/state)."""
import json
import os
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "pulsar-tlaplus_amd", "python"))
sys.path.insert(0, ROOT)
import tlcgpu as T  # noqa: E402
from bench import CONFIGS, model_for  # noqa: E402

base_env = dict(os.environ)
reps = int(os.environ.get("PROBE_REPS", "3"))
for spec in sys.argv[1:]:
    parts = spec.split("|")
    head = parts[0].split(":")
    name, cfg = head[0], head[1]
    rank, world = (int(x) for x in head[2].split("/")) if len(head) > 2 else (0, 1)
    envs = parts[1] if len(parts) > 1 else ""
    defs = parts[2] if len(parts) > 2 else ""
    os.environ.clear()
    os.environ.update(base_env)
    for kv in filter(None, envs.replace("+", ",").split(",")):  # ('+' too: gpu.sh splits cases on ',')
        k, v = kv.split("=", 1)
        os.environ[k] = v
    if defs:
        os.environ["TLCG_JIT_DEFINES"] = defs
    c = CONFIGS[cfg]
    m = model_for(cfg)
    t0 = time.perf_counter()
    eng = os.environ.get("PROBE_ENGINE", "auto")  # (global: the HBM-FPSet engine, pre-sized)
    log2 = max(16, (2 * (c["distinct"] // world + 1) - 1).bit_length()) if eng == "global" else 0
    ck = T.Checker(m, rank=rank, world=world, engine=eng, log2_fpset_slots=log2,
                   tlc_order=os.environ.get("PROBE_TLC", "0") == "1",
                   state_capacity=int(c["distinct"] * 1.15 / world) + (1 << 20))
    best, walls = 1e9, []
    for _ in range(reps):
        w0 = time.perf_counter()
        st = ck.run_raw()
        walls.append((time.perf_counter() - w0) * 1e3)
        best = min(best, st.kernel_ms)
    d = st.distinct
    ok = (st.generated, d) == (c["generated"], c["distinct"]) if world == 1 else None
    ck.close()
    print(json.dumps(dict(case=spec, cfg=cfg, rank=rank, world=world, kernel_ms=round(best, 4),
                          wall_ms=round(min(walls), 3), distinct=d, generated=st.generated, counts_ok=ok,
                          ps_per_state=round(best * 1e9 / max(d, 1), 3),
                          engine=T.ENGINE_NAMES.get(int(st.engine), "?"), jit=int(st.jit_used),
                          setup_s=round(time.perf_counter() - t0, 1))), flush=True)
