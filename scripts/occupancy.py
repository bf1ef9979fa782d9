"""Occupancy experiment: components of 18 states (C=1, K=1), on-chip capacity 32 vs 64."""
import os, sys, time, json
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'pulsar-tlaplus_amd', 'python'))
import tlcgpu as T
m = T.Model(key_space=range(1, 16), value_space=range(1, 16), compaction_times_limit=1)
os.environ["TLCG_JIT"] = "1"
for k0 in ("64", "32"):
    os.environ["TLCG_COMP_K0"] = k0
    ck = T.Checker(m, engine="component")
    best = 1e9
    for rep in range(4):
        st = ck.run_raw()
        best = min(best, st.kernel_ms)
    print(json.dumps(dict(k0=k0, distinct=st.distinct, generated=st.generated, kernel_ms=round(best, 2),
                          states_per_s=st.distinct / best * 1e3)), flush=True)
    ck.close()
