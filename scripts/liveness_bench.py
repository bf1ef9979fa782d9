"""PROPERTY Termination (compaction.tla:303-307) on the GPU at scale:
tlcg_check_termination on a scaled cfg under Spec and Spec /\\ WF_vars(Next),
counts checked against the per-component law (SURVEY App.A.1: S's 57 not-P
states and 71 edges per initial message sequence).  One JSON line per run.
Usage: python scripts/liveness_bench.py [keys=15] [reps=3]"""
import json, os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'pulsar-tlaplus_amd', 'python'))
import tlcgpu as T
keys = int(sys.argv[1]) if len(sys.argv) > 1 else 15
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
m = T.Model(key_space=range(1, keys + 1), value_space=range(1, keys + 1))
n_init = (keys + 1) ** 6
for fair in ("wf", "none"):
    best = None
    calls = []
    for _ in range(reps):
        t0 = time.perf_counter()
        lv = T.check_termination(m, fair, state_capacity=57 * n_init + 1024)
        wall = time.perf_counter() - t0
        calls.append(round(lv.wall_ms, 1))
        assert (lv.states_notp, lv.edges_notp, lv.init_notp) == (57 * n_init, 71 * n_init, n_init), lv
        assert lv.holds == (fair == "wf")
        if best is None or lv.kernel_ms < best[0].kernel_ms:
            best = (lv, wall)
    lv, wall = best
    print(json.dumps(dict(cfg=f"KeySpace = ValueSpace = 1..{keys}", fairness=fair, holds=lv.holds, kind=lv.kind,
                          states_notp=lv.states_notp, edges_notp=lv.edges_notp, peel_rounds=lv.peel_rounds,
                          kernel_ms=round(lv.kernel_ms, 2), call_ms=round(lv.wall_ms, 1), call_ms_reps=calls,
                          states_per_s=round(lv.states_notp / (lv.kernel_ms * 1e-3), 1),
                          trace_len=len(lv.trace))), flush=True)
