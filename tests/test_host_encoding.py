"""CPU: the product's packed encoding (model.h, compiled for the host inside
libtlcgpu.so -- the same code the gfx950 kernels run) against the oracle.

A plain Python BFS over tlcg_host_successors must reproduce the golden counts,
per-level sizes and traces; decoded trace states must match the oracle's TLC
text byte for byte.  No GPU call is made."""
import ctypes

import pytest

import tlcgpu
from conftest import FULL_CASES, GOLDEN, model_of


def host_bfs(m):
    n = tlcgpu.init_count(m)
    seen, order, parent, act = {}, [], [], []
    for i in range(n):
        s = tlcgpu.host_init_state(m, i)
        seen[s] = len(order)
        order.append(s)
        parent.append(-1)
        act.append("Init")
        c = tlcgpu.host_check_invariants(m, s)
        if c >= 0:
            return dict(result="invariant", invariant=m.invariants[c >> 1], trace=[("Init", s)])
    gen, levels, head = n, [n] if n else [], 0

    def trace_to(k):
        out = []
        while k >= 0:
            out.append((act[k], order[k]))
            k = parent[k]
        return out[::-1]

    while head < len(order):
        end = len(order)
        for p in range(head, end):
            succ = tlcgpu.host_successors(m, order[p])
            if not succ and m.check_deadlock:
                return dict(result="deadlock", trace=trace_to(p))
            for a, t in succ:
                gen += 1
                if t not in seen:
                    seen[t] = len(order)
                    order.append(t)
                    parent.append(p)
                    act.append(a)
                    c = tlcgpu.host_check_invariants(m, t)
                    if c >= 0:
                        return dict(result="invariant", invariant=m.invariants[c >> 1], trace=trace_to(len(order) - 1))
        head = end
        if len(order) > end:
            levels.append(len(order) - end)
    return dict(result="ok", generated=gen, distinct=len(order), depth=len(levels), levels=levels)


CASES = ["S", "S_noretain", "S_consumer", "S_consumer_ctl0", "V_leak", "V_dup", "V_dup_producer", "D_N0_K1",
         "D_N0_K0", "D_N0_K1_nodeadlock", "X_keys3_vals57", "X_producer_sparse", "X_C5_K2", "X_empty_spaces",
         "R_C6_K3", "R_C1_K0"]


@pytest.mark.parametrize("case", CASES)
def test_host_encoding_bfs(case):
    g = GOLDEN[case]
    m = model_of(g["constants"])
    r = host_bfs(m)
    want = g["result"]
    assert r["result"] == want["result"]
    if want["result"] == "ok":
        assert (r["generated"], r["distinct"], r["depth"], r["levels"]) == (
            want["generated"], want["distinct"], want["depth"], want["levels"])
    else:
        assert [a for a, _ in r["trace"]] == [t["action"] for t in want["trace"]]
        assert [tlcgpu.decode(m, s) for _, s in r["trace"]] == [t["state"] for t in want["trace"]]
        if want["result"] == "invariant":
            assert r["invariant"] == want["invariant"]


def test_host_encoding_published_producer():
    # compaction.tla:23: 253361 with the producer modelled (RetainNullKey = FALSE)
    r = host_bfs(model_of(GOLDEN["P_published"]["constants"]))
    assert r["distinct"] == 253361 and r["generated"] == GOLDEN["P_published"]["result"]["generated"]


def test_state_bits():
    assert tlcgpu.state_bits(tlcgpu.Model()) == 41
    g9 = tlcgpu.Model(key_space=range(1, 16), value_space=range(1, 16))
    assert tlcgpu.state_bits(g9) == 53  # SURVEY App.B: 55 with the (constant) consumeTimes field
    assert tlcgpu.init_count(g9) == 16 ** 6


def test_init_order_first_is_all_null():
    m = tlcgpu.Model()
    assert tlcgpu.decode(m, tlcgpu.host_init_state(m, 0)).startswith(
        "/\\ messages = <<[id |-> 1, key |-> 0, value |-> 0], [id |-> 2, key |-> 0, value |-> 0]")
    # message 1 varies fastest, its key faster than its value
    assert "[id |-> 1, key |-> 1, value |-> 0]" in tlcgpu.decode(m, tlcgpu.host_init_state(m, 1))
    assert "[id |-> 1, key |-> 0, value |-> 1]" in tlcgpu.decode(m, tlcgpu.host_init_state(m, 3))
    assert "[id |-> 2, key |-> 1, value |-> 0]" in tlcgpu.decode(m, tlcgpu.host_init_state(m, 9))


def test_phase_one_result_printing():
    m = tlcgpu.Model(key_space=[2, 5], value_space=[1])
    s = tlcgpu.host_init_state(m, 1 + 3 * 0 + 6 * 2)  # msg1 key 2, msg2 key 5
    (a, t), = [x for x in tlcgpu.host_successors(m, s) if x[0] == "CompactorPhaseOne"]
    txt = tlcgpu.decode(m, t)
    assert "phaseOneResult = [latestForKey |-> (2 :> 1 @@ 5 :> 2), readPosition |-> 3]" in txt


@pytest.mark.parametrize("case", [c for c in FULL_CASES if not GOLDEN[c]["constants"]["producer"]])
def test_component_specialization_matches_generic(case):
    """component_model.h (messages-hoisted evaluators of the component engine)
    agrees with model.h on every state of the first components of each
    golden cfg: compactor successor, stutter count, first failing invariant."""
    m = model_of(GOLDEN[case]["constants"])
    n = tlcgpu.host_component_selfcheck(m, 0, 300)
    bits = tlcgpu.load_library().tlcg_state_bits(m.to_c())
    assert n > 0 or (n == 0 and bits > 32), n


def test_horizon_correctness_retained_null_key_takes_else_branch():
    """CompactionHorizonCorrectness (compaction.tla:262-274) read literally:
    with RetainNullKey = TRUE, messagesBeforeHorizon[i] of a null-key message
    is the message itself, never Nil, so the ELSE branch applies -- some ledger
    entry with key 0 and id >= i witnesses it.  A ledger holding message 2 (a
    null key) but not message 1 (also a null key) therefore satisfies i = 1.
    "The same record must be in the ledger" would say FALSE here; the two
    readings differ only off the reachable space (reachable ledgers keep every
    null-key message up to their read position)."""
    import oracle_py
    m = tlcgpu.Model()  # S: RetainNullKey = TRUE, invariants TypeSafe, CompactionHorizonCorrectness
    s = tlcgpu.host_init_state(m, 81)  # <<(1, key 0), (2, key 0), (3, key 1)>>
    for _ in range(4):  # PhaseOne, Write, UpdateContext, UpdateHorizon: hz = 3, ctx = 1
        s = [t for a, t in tlcgpu.host_successors(m, s) if a != "BrokerCrash"][0]
    assert tlcgpu.host_check_invariants(m, s) == -1
    full = "<<<<[id |-> 1, key |-> 0, value |-> 0], [id |-> 2, key |-> 0, value |-> 0], [id |-> 3, key |-> 1, value |-> 0]>>, Nil, Nil>>"
    want = "<<<<[id |-> 2, key |-> 0, value |-> 0], [id |-> 3, key |-> 1, value |-> 0]>>, Nil, Nil>>"
    assert full in tlcgpu.decode(m, s)
    # the word whose ledger 1 lacks message 1: one flipped bit of the packed state
    v, = [s ^ (1 << b) for b in range(tlcgpu.state_bits(m)) if want in tlcgpu.decode(m, s ^ (1 << b))]
    assert "compactionHorizon = 3" in tlcgpu.decode(m, v) and "compactedTopicContext = 1" in tlcgpu.decode(m, v)
    assert tlcgpu.host_check_invariants(m, v) == -1  # the ELSE branch holds for i = 1 (entry 2: key 0, id 2 >= 1)
    # the Python oracle on the same TLC values
    py = oracle_py.Model(N=3, C=3, K=1, keys=[1, 2], values=[1, 2], retain=True, producer=False, consumer=False, ctl=2)
    msgs = ((1, 0, 0), (2, 0, 0), (3, 1, 0))
    state = (msgs, (msgs[1:], None, None), None, oracle_py.W + 3, None, 3, 1, 0, 0)
    assert py.inv("CompactionHorizonCorrectness", state) is True
    # drop message 2 as well: no entry with key 0 remains, i = 1 fails
    state = (msgs, (msgs[2:], None, None), None, oracle_py.W + 3, None, 3, 1, 0, 0)
    assert py.inv("CompactionHorizonCorrectness", state) is False
    w = v ^ next(1 << b for b in range(tlcgpu.state_bits(m))
                 if "<<<<[id |-> 3, key |-> 1, value |-> 0]>>, Nil, Nil>>" in tlcgpu.decode(m, v ^ (1 << b)))
    assert tlcgpu.host_check_invariants(m, w) == (1 << 1)  # index 1 (CompactionHorizonCorrectness), false
    # the component engine's specialized evaluators agree on such words too
    # (tlcg_host_component_selfcheck flips every ledger bit of every state)
    assert tlcgpu.host_component_selfcheck(m, 81, 1) > 0


@pytest.mark.parametrize("case", ["S", "P_published", "S_consumer", "W_C12_k1", "D_N0_K0", "X_empty_spaces"])
def test_termination_counterexample(case):
    """PROPERTY Termination: Spec has no fairness, so <>P fails iff an initial
    state violates P (the behavior: that state, then stuttering).  The first
    such state in Init order, against the Python oracle's P."""
    import oracle_py
    c = GOLDEN[case]["constants"]
    m = model_of(c)
    py = oracle_py.Model(N=c["N"], C=c["C"], K=c["K"], keys=c["keys"], values=c["values"], retain=c["retain"],
                         producer=c["producer"], consumer=c["consumer"], ctl=c["ctl"])

    def p(s):  # the body of Termination, compaction.tla:303-307
        msgs, led, cur, ph, p1r, hz, ctx, crash, cons = s
        return (len(msgs) == c["N"] and ph == oracle_py.W and py.max_ledger(led) == c["C"]
                and (not c["consumer"] or cons == c["ctl"]))
    want = next((i for i, s in enumerate(py.inits()) if not p(s)), -1)
    lib = tlcgpu.load_library()
    lib.tlcg_host_termination_counterexample.restype = ctypes.c_int64
    got = lib.tlcg_host_termination_counterexample(ctypes.byref(m.to_c()))
    assert got == want == 0  # every initial state is in PhaseOne (compaction.tla:199)
