"""G9 on the global engine with the state store resident in HBM vs spilled to
pinned host memory (tlcg_opts.spill with a device store cap), and with the
host FPSet tier (tlcg_opts.fpset_spill with the HBM table capped).  Count-checked;
prints one JSON line per mode."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'pulsar-tlaplus_amd', 'python'))
import tlcgpu as T

m = T.Model(key_space=range(1, 16), value_space=range(1, 16))
cap = int(sys.argv[1]) if len(sys.argv) > 1 else 200_000_000
tier = int(sys.argv[2]) if len(sys.argv) > 2 else 28
modes = (("resident", dict(state_capacity=1_200_000_000, log2_fpset_slots=31)),
         ("spill", dict(spill=True, device_store_cap=cap, log2_fpset_slots=31)),
         ("fpset_tier", dict(state_capacity=1_200_000_000, fpset_spill=True, log2_fpset_max=tier)),
         ("spill+fpset_tier", dict(spill=True, device_store_cap=cap, fpset_spill=True, log2_fpset_max=tier)))
for name, kw in modes:
    ck = T.Checker(m, engine="global", **kw)
    walls = []
    for rep in range(3):
        t = time.perf_counter()
        st = ck.run_raw()
        walls.append(time.perf_counter() - t)
        assert (st.generated, st.distinct, st.depth) == (1392508928, 1040187392, 20), (st.generated, st.distinct)
    # a trace-style read of the oldest (spilled) states
    t = time.perf_counter()
    first = ck.copy_states(0, 1 << 20)
    read_s = time.perf_counter() - t
    ck.close()
    print(json.dumps(dict(mode=name, device_store_cap=kw.get("device_store_cap", 0), wall_s=[round(w, 3) for w in walls],
                          kernel_ms=round(st.kernel_ms, 1), expand_ms=round(st.expand_ms, 1),
                          host_states=st.host_states, fpset_host_states=st.fpset_host_states,
                          distinct=st.distinct,
                          distinct_per_s=round(st.distinct / min(walls), 0),
                          read_1M_states_ms=round(read_s * 1e3, 1), first_state=first[0])), flush=True)
