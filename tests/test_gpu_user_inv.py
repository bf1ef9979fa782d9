"""GPU: whole checks with user invariants (BASELINE config 5: an invariant
injected into compaction.tla, violated at depth) against the Python oracle's
fixtures (tests/golden/user_inv.json, oracle/tla_eval.py): verdict, the
violated invariant, depth, counts, TLC's counterexample trace text and TLC's
counters at its stop point.  The invariants run in k_user_check on the GPU."""
import json
import os

import pytest

import tlcgpu

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = json.load(open(os.path.join(HERE, "golden", "user_inv.json")))


def model(case):
    g = GOLD[case]
    return tlcgpu.Model(invariants=tuple(g["invariants"]), user_defs=g["user_defs"], **g["constants"])


@pytest.mark.parametrize("order", ["tlc_order", "fast"])
@pytest.mark.parametrize("case", sorted(GOLD))
def test_user_invariant_check(case, order):
    m = model(case)
    want = GOLD[case]["result"]
    ck = tlcgpu.Checker(m, tlc_order=order == "tlc_order")
    r = ck.run()
    assert r.engine == "global"
    assert r.status == want["result"], (case, r.status)
    if want["result"] == "ok":
        assert (r.generated, r.distinct, r.depth, r.levels) == (want["generated"], want["distinct"], want["depth"],
                                                                 want["levels"])
        return
    # the run finishes the level that found the error (end-of-level counts), the trace is TLC's
    assert r.depth == want["depth"]
    assert (r.generated, r.distinct) == (want["eol_generated"], want["eol_distinct"])
    if want["result"] in ("invariant", "invariant_error"):
        assert r.invariant == want["invariant"]
    if order == "tlc_order":
        assert [a for a, _ in r.trace] == [t["action"] for t in want["trace"]]
        assert [tlcgpu.decode(m, s) for _, s in r.trace] == [t["state"] for t in want["trace"]]
        # TLC's "X states generated, Y distinct states found, Z states left on queue" at its stop
        assert ck.tlc_stop_stats() == (want["generated"], want["distinct"], want["left_on_queue"])
    else:
        # some shortest counterexample: a path of the spec ending in a violating state
        assert r.trace[0][0] == "Init" and len(r.trace) == want["depth"]
        for (_, s), (a, t) in zip(r.trace, r.trace[1:]):
            assert (a, t) in tlcgpu.host_successors(m, s)
        c = tlcgpu.host_check_invariants(m, r.trace[-1][1])
        assert c >= 0 and m.invariants[c >> 1] == want["invariant"]
    ck.close()


def test_user_invariants_refuse_other_engines_and_ranks():
    m = model("U_LedgerCount")
    for kw in (dict(engine="component"), dict(engine="tree"), dict(world=2)):
        with pytest.raises(RuntimeError):
            tlcgpu.Checker(m, **kw)


def test_user_invariant_at_scale():
    """M8 (1.1e8 states) with an invariant that holds everywhere and one that
    fails at depth 12: the check kernel runs on every level of the global engine"""
    g = GOLD["U_all_hold"]
    keys = range(1, 11)
    m = tlcgpu.Model(key_space=keys, value_space=keys, invariants=tuple(g["invariants"]), user_defs=g["user_defs"])
    r = tlcgpu.Checker(m, state_capacity=120_000_000).run(with_trace=False)
    assert (r.status, r.generated, r.distinct, r.depth) == ("ok", 147_039_563, 109_836_782, 20)
    g = GOLD["U_LedgerCount"]
    m = tlcgpu.Model(key_space=keys, value_space=keys, invariants=tuple(g["invariants"]), user_defs=g["user_defs"])
    r = tlcgpu.Checker(m, tlc_order=True, state_capacity=120_000_000).run()
    assert (r.status, r.invariant, r.depth) == ("invariant", "LedgerCount", 12)
    # the per-message-sequence law (SURVEY App.A.1): every component reaches the same depth-12 level
    assert r.distinct % tlcgpu.init_count(m) == 0
