"""Sweep k_expand variants on the G9 config (tuning; every run is count-checked)."""
import os, sys, time, json
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'pulsar-tlaplus_amd', 'python'))
import tlcgpu as T
cfg = sys.argv[1] if len(sys.argv) > 1 else "g9"
k = 15 if cfg == "g9" else 10
m = T.Model(key_space=range(1, k + 1), value_space=range(1, k + 1))
want = (1392508928, 1040187392) if k == 15 else (147039563, 109836782)
variants = [dict(TLCG_FAST_ITEMS="0")]
for it in ("1", "2", "4"):
    for pr in ("0", "1"):
        variants.append(dict(TLCG_FAST_ITEMS=it, TLCG_PROBE=pr))
variants += [dict(TLCG_FAST_ITEMS="2", TLCG_PROBE="0", TLCG_GRID=g) for g in ("2048", "4096", "16384", "65536")]
for v in variants:
    for key in ("TLCG_FAST_ITEMS", "TLCG_PROBE", "TLCG_GRID"):
        os.environ.pop(key, None)
    os.environ.update(v)
    ck = T.Checker(m, log2_fpset_slots=31 if k == 15 else 28, state_capacity=1_200_000_000 if k == 15 else 130_000_000)
    best = None
    for rep in range(3):
        t = time.perf_counter(); st = ck.run_raw(); wall = time.perf_counter() - t
        assert (st.generated, st.distinct) == want, (st.generated, st.distinct)
        r = (wall * 1e3, st.expand_ms, st.kernel_ms)
        best = r if best is None or r[0] < best[0] else best
    ck.close()
    print(json.dumps(dict(variant=v, wall_ms=round(best[0], 2), expand_ms=round(best[1], 2), kernel_ms=round(best[2], 2))), flush=True)
