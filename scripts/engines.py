"""G9 wall/kernel time per engine and kernel flavour (tuning; count-checked)."""
import os, sys, time, json
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'pulsar-tlaplus_amd', 'python'))
import tlcgpu as T
m = T.Model(key_space=range(1, 16), value_space=range(1, 16))
which = sys.argv[1] if len(sys.argv) > 1 else "all"
runs = (("component", "1"), ("component", "0"), ("global", "0")) if which == "all" else (("component", "1"),)
for eng, jit in runs:
    os.environ["TLCG_JIT"] = jit
    t0 = time.perf_counter()
    ck = T.Checker(m, engine=eng, state_capacity=1_200_000_000, log2_fpset_slots=31 if eng == "global" else 0)
    best = None
    for rep in range(4):
        t = time.perf_counter(); st = ck.run_raw(); wall = time.perf_counter() - t
        if rep == 0: first = wall
        assert (st.generated, st.distinct) == (1392508928, 1040187392), (st.generated, st.distinct)
        r = (wall * 1e3, st.expand_ms, st.kernel_ms, int(st.jit_used))
        best = r if best is None or r[0] < best[0] else best
    ck.close()
    print(json.dumps(dict(engine=eng, jit=best[3], first_run_s=round(first, 3), wall_ms=round(best[0], 2),
                          expand_ms=round(best[1], 2), kernel_ms=round(best[2], 2))), flush=True)
