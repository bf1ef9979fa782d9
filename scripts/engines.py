"""G9 wall/kernel time per engine (tuning; count-checked)."""
import os, sys, time, json
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'pulsar-tlaplus_amd', 'python'))
import tlcgpu as T
m = T.Model(key_space=range(1, 16), value_space=range(1, 16))
for eng in ("component", "global"):
    ck = T.Checker(m, engine=eng, state_capacity=1_200_000_000, log2_fpset_slots=31 if eng == "global" else 0)
    best = None
    for rep in range(4):
        t = time.perf_counter(); st = ck.run_raw(); wall = time.perf_counter() - t
        assert (st.generated, st.distinct) == (1392508928, 1040187392), (st.generated, st.distinct)
        r = (wall * 1e3, st.expand_ms, st.kernel_ms)
        best = r if best is None or r[0] < best[0] else best
    ck.close()
    print(json.dumps(dict(engine=eng, wall_ms=round(best[0], 2), expand_ms=round(best[1], 2), kernel_ms=round(best[2], 2))), flush=True)
