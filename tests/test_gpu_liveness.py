"""GPU: PROPERTY Termination (compaction.tla:303-307) checked by the HIP
liveness pass (tlcg_check_termination, csrc/liveness.hip) against the golden
liveness results of the oracles -- the C oracle's Tarjan SCC restatement,
cross-checked with the Python oracle's DFS (tests/golden/make_golden.py) --
under Spec (no fairness, compaction.tla:233) and Spec /\\ WF_vars(Next).

What is pinned: holds / fails, |G'| (the states reachable from Init through
not-P states), its initial states and edges, the states where a behavior may
stutter forever, and the depth of the shallowest one.  Which counterexample is
printed is [TLC-ext]: the test checks that the returned one is a behavior of
the spec that never reaches P and ends where the fairness allows stuttering."""
import pytest

import tlcgpu
from conftest import GOLDEN, model_of

pytestmark = pytest.mark.gpu

LIVE_CASES = sorted(k for k, v in GOLDEN.items() if "liveness" in v)
G9 = dict(key_space=range(1, 16), value_space=range(1, 16))


def is_p(m, s):
    """Termination's predicate P: the guard of Terminating (:205-214), i.e.
    Terminating is among the state's successors (it needs P and nothing else)"""
    return any(a == "Terminating" for a, _ in tlcgpu.host_successors(m, s))


def check_counterexample(m, lv):
    assert lv.kind == "stuttering" and lv.loop_to == -1
    tr = lv.trace
    assert tr and tr[0][0] == "Init"
    assert tr[0][1] in {tlcgpu.host_init_state(m, i) for i in range(tlcgpu.init_count(m))}
    for (_, s), (a, t) in zip(tr, tr[1:]):
        assert (a, t) in tlcgpu.host_successors(m, s)
    assert not any(is_p(m, s) for _, s in tr)
    if lv.fairness == "wf":  # <<Next>>_vars disabled at the end: every successor is a stutter
        last = tr[-1][1]
        assert all(t == last for _, t in tlcgpu.host_successors(m, last))


@pytest.mark.parametrize("fair", ["none", "wf"])
@pytest.mark.parametrize("case", LIVE_CASES)
def test_termination_golden(case, fair):
    want = GOLDEN[case]["liveness"][fair]
    m = model_of(GOLDEN[case]["constants"])
    lv = tlcgpu.check_termination(m, fair)
    assert lv.holds == want["holds"], (case, fair)
    assert (lv.states_notp, lv.init_notp, lv.edges_notp, lv.stuck) == \
           (want["states_notp"], want["init_notp"], want["edges_notp"], want["stuck"]), (case, fair)
    assert (lv.on_cycles == 0) == (want["cyclic_sccs"] == 0)
    if want["holds"]:
        assert lv.kind == "holds" and lv.trace == []
        return
    check_counterexample(m, lv)
    if fair == "none":
        # Spec has no fairness: the first not-P initial state in Init order, then
        # stuttering -- the same state as the host closed form
        assert len(lv.trace) == 1
        assert lv.trace[0][1] == tlcgpu.host_init_state(m, tlcgpu.load_library().tlcg_host_termination_counterexample(
            m.to_c()))
    else:
        assert len(lv.trace) == want["stuck_min_depth"]  # a shallowest stuck state


def test_termination_regrows():
    """a store / FPSet far too small for G' is grown and the BFS redone"""
    m = model_of(GOLDEN["S_consumer"]["constants"])
    want = GOLDEN["S_consumer"]["liveness"]["wf"]
    lv = tlcgpu.check_termination(m, "wf", state_capacity=100, log2_fpset_slots=8)
    assert (lv.holds, lv.states_notp, lv.edges_notp, lv.stuck) == \
           (False, want["states_notp"], want["edges_notp"], want["stuck"])
    assert len(lv.trace) == want["stuck_min_depth"]


def test_termination_wide_states():
    """a > 63-bit layout (CompactionTimesLimit = 12): two-word states through
    the wide FPSet"""
    case = "W_C12_k1"
    m = model_of(GOLDEN[case]["constants"])
    assert tlcgpu.state_words(m) == 2
    for fair in ("none", "wf"):
        want = GOLDEN[case]["liveness"][fair]
        lv = tlcgpu.check_termination(m, fair)
        assert (lv.holds, lv.states_notp, lv.edges_notp, lv.stuck) == \
               (want["holds"], want["states_notp"], want["edges_notp"], want["stuck"])


def test_termination_g9_scaled():
    """G9 (~1e9 reachable states): components are isomorphic (SURVEY App.A.1),
    so G' is 16^6 times S's per-component figures: 57 not-P states and 71 edges
    per initial message sequence; under WF_vars(Next) no stuck state and no
    cycle, so Termination holds; without fairness it fails at the first
    initial state."""
    m = tlcgpu.Model(**G9)
    s = GOLDEN["S"]["liveness"]["wf"]
    per_state, per_edge = s["states_notp"] // 729, s["edges_notp"] // 729
    assert (per_state, per_edge) == (57, 71)
    lv = tlcgpu.check_termination(m, "wf", state_capacity=16 ** 6 * per_state + 1024)
    assert lv.holds and lv.kind == "holds"
    assert (lv.states_notp, lv.init_notp, lv.edges_notp, lv.stuck, lv.on_cycles) == \
           (16 ** 6 * per_state, 16 ** 6, 16 ** 6 * per_edge, 0, 0)
    print(f"G9 Termination under WF_vars(Next): {lv.states_notp} states, {lv.edges_notp} edges, "
          f"{lv.peel_rounds} peel rounds, kernels {lv.kernel_ms:.1f} ms, call {lv.wall_ms:.1f} ms")
