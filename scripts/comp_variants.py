"""Tuning: G9 component-kernel time under hipRTC define sets (TLCG_JIT_DEFINES);
each variant is count-checked.  Usage: python scripts/comp_variants.py "" "A=1;B" ...
A variant "ENV=V,ENV2=V|defines" also sets environment variables (e.g. "TLCG_CODE=0|")."""
import json, os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'pulsar-tlaplus_amd', 'python'))
import tlcgpu as T
keys = int(os.environ.get("VKEYS", "15"))
m = T.Model(key_space=range(1, keys + 1), value_space=range(1, keys + 1))
os.environ["TLCG_JIT"] = "1"
base_env = dict(os.environ)
for spec in sys.argv[1:] or [""]:
    envs, defs = spec.split("|", 1) if "|" in spec else ("", spec)
    os.environ.clear()
    os.environ.update(base_env)
    for kv in filter(None, envs.split(",")):
        k, v = kv.split("=", 1)
        os.environ[k] = v
    os.environ["TLCG_JIT_DEFINES"] = defs
    t0 = time.perf_counter()
    ck = T.Checker(m, engine="component", state_capacity=int(1.1 * 62 * (keys + 1) ** 6))
    best = 1e9
    for rep in range(3):
        st = ck.run_raw()
        best = min(best, st.kernel_ms)
    ok = (st.generated, st.distinct) == (1392508928, 1040187392) if keys == 15 else None
    ck.close()
    print(json.dumps(dict(variant=spec, defines=defs, kernel_ms=round(best, 3), counts_ok=ok, jit=int(st.jit_used),
                          setup_s=round(time.perf_counter() - t0, 1))), flush=True)
