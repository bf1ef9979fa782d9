"""GPU: whole checks with user invariants (BASELINE config 5: an invariant
injected into compaction.tla, violated at depth) against the Python oracle's
fixtures (tests/golden/user_inv.json, oracle/tla_eval.py): verdict, the
violated invariant, depth, counts, TLC's counterexample trace text and TLC's
counters at its stop point.  The global engine runs them in its level check
(tlcg_user_check, generated device code; k_user_check interprets with TLCG_JIT=0);
the on-chip engines (component, component tree) run them as device code
generated from the compiled program (user_inv.cpp user_device_source) inside
their hipRTC-specialized kernels; the ranks of a multi-GPU check run them in
whichever engine each rank uses."""
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


def check_path(m, r, want):
    """some shortest counterexample: a path of the spec ending in a violating state"""
    assert r.trace[0][0] == "Init" and len(r.trace) == want["depth"]
    for (_, s), (a, t) in zip(r.trace, r.trace[1:]):
        assert (a, t) in tlcgpu.host_successors(m, s)
    c = tlcgpu.host_check_invariants(m, r.trace[-1][1])
    assert c >= 0 and m.invariants[c >> 1] == want["invariant"]


@pytest.mark.parametrize("order", ["tlc_order", "fast"])
@pytest.mark.parametrize("case", sorted(GOLD))
def test_user_invariant_check(case, order):
    """the global engine (TLC order, or forced): k_user_check on every level"""
    m = model(case)
    want = GOLD[case]["result"]
    ck = tlcgpu.Checker(m, tlc_order=order == "tlc_order", engine="global")
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
        check_path(m, r, want)
    ck.close()


@pytest.mark.parametrize("jit", ["0", "1"])
@pytest.mark.parametrize("case", ["U_LedgerCount", "U_all_hold", "U_ContextLedgerError", "U_mixed_user_first",
                                  "U_producer_LedgerCount"])
def test_user_invariant_global_check_kernel(case, jit, monkeypatch):
    """the global engine's level check as hipRTC device code (tlcg_user_check,
    jit_used bit 2) and as the interpreter (TLCG_JIT=0, k_user_check): the
    same verdict, counts and TLC-order stop point"""
    monkeypatch.setenv("TLCG_JIT", jit)
    m = model(case)
    want = GOLD[case]["result"]
    ck = tlcgpu.Checker(m, tlc_order=True, engine="global")
    st = ck.run_raw()
    assert bool(st.jit_used & 4) == (jit == "1")
    r = ck.run()
    assert r.status == want["result"] and r.depth == want["depth"]
    if want["result"] == "ok":
        assert (r.generated, r.distinct) == (want["generated"], want["distinct"])
    else:
        assert (r.generated, r.distinct) == (want["eol_generated"], want["eol_distinct"])
        assert ck.tlc_stop_stats() == (want["generated"], want["distinct"], want["left_on_queue"])


# the on-chip engines' first-pass kernels (tests/test_gpu_wave_parity.py): the
# default (one walk per wavefront), the per-lane bitmap pass (component_lane.h)
# and the per-lane pass of component_body.h
KERNELS = {"default": {}, "perlane": {"TLCG_COMP_WAVE": "0", "TLCG_TREE_WAVE": "0"},
           "perlane_body": {"TLCG_COMP_WAVE": "0", "TLCG_TREE_WAVE": "0", "TLCG_COMP_LANE": "0"}}


@pytest.mark.parametrize("case", ["U_LedgerCount", "U_all_hold", "U_ContextLedgerError", "U_mixed_user_first",
                                  "U_noretain_LatestIsLast"])
def test_user_invariant_global_fast_specialized(case, monkeypatch):
    """the global engine in fast order with the layout-specialized expand
    (expand_fast.h, jit_used bit 6; TLCG_JIT=1 forces it on these small
    models): the expand kernel leaves the user invariants to the level's
    check kernel (Layout.defer_inv, which the specialized layout must carry),
    so the verdict, depth and end-of-level counts are the fixture's"""
    monkeypatch.setenv("TLCG_JIT", "1")
    m = model(case)
    want = GOLD[case]["result"]
    ck = tlcgpu.Checker(m, engine="global")
    try:
        r = ck.run()
        assert r.jit_used & 64 and r.jit_used & 4, r.jit_used
        assert r.status == want["result"] and r.depth == want["depth"], (case, r.status, r.depth)
        if want["result"] == "ok":
            assert (r.generated, r.distinct) == (want["generated"], want["distinct"])
        else:
            assert (r.generated, r.distinct) == (want["eol_generated"], want["eol_distinct"])
            assert r.invariant == want.get("invariant", r.invariant)
    finally:
        ck.close()


@pytest.mark.parametrize("kernel", sorted(KERNELS))
@pytest.mark.parametrize("case", sorted(GOLD))
def test_user_invariant_on_chip(case, kernel, monkeypatch):
    """the default engine with the user invariants inside its specialized
    kernels: the component engine without a Producer (its lanes keep TLC's
    order), the component tree's closed mode past a lane's 255 states (its
    error replayed in TLC's order on the host), the component tree with a
    Producer (its error reported by the global engine in TLC order); every
    error's trace and TLC's stop counters are TLC's, with no second run"""
    for k, v in KERNELS[kernel].items():
        monkeypatch.setenv(k, v)
    m = model(case)
    want = GOLD[case]["result"]
    # (C = 5: the local key passes 32 bits, or 302 states per component at K = 2: the tree's closed mode)
    on_chip = "tree" if m.model_producer or case.startswith("U_C5") else "component"
    ck = tlcgpu.Checker(m)
    r = ck.run()
    assert r.status == want["result"], (case, r.status)
    if want["result"] == "ok":
        assert r.engine == on_chip
        assert (r.generated, r.distinct, r.depth, r.levels) == (want["generated"], want["distinct"], want["depth"],
                                                                 want["levels"])
        ck.close()
        return
    assert r.engine == on_chip and r.tlc_exact
    assert r.depth == want["depth"]
    assert (r.generated, r.distinct) == (want["eol_generated"], want["eol_distinct"])
    if want["result"] in ("invariant", "invariant_error"):
        assert r.invariant == want["invariant"]
    assert [a for a, _ in r.trace] == [t["action"] for t in want["trace"]]
    assert [tlcgpu.decode(m, s) for _, s in r.trace] == [t["state"] for t in want["trace"]]
    assert ck.tlc_stop_stats() == (want["generated"], want["distinct"], want["left_on_queue"])
    ck.close()


@pytest.mark.parametrize("utab", ["0", "dyn", "slow"])
@pytest.mark.parametrize("case", ["U_LedgerCount", "U_all_hold", "U_ContextLedgerError", "U_mixed_user_first",
                                  "U_noretain_LatestIsLast", "U_C5_ContextBound"])
@pytest.mark.parametrize("kernel", ["default", "perlane"])
def test_user_invariant_outcome_tables(case, utab, kernel, monkeypatch):
    """the outcome tables (component_code.h code_consts_user) against the
    programs: no tables (TLCG_UTAB=0), tables filled per component only
    (dyn), and every entry left to the kernel's fallback evaluation (slow)
    give the same verdict, counts, trace and stop counters as the default
    (host-made class tables + per-component ones) -- the golden fixture"""
    monkeypatch.setenv("TLCG_UTAB", utab)
    for k, v in KERNELS[kernel].items():
        monkeypatch.setenv(k, v)
    m = model(case)
    want = GOLD[case]["result"]
    ck = tlcgpu.Checker(m)
    r = ck.run()
    assert r.status == want["result"], (case, utab, r.status)
    if want["result"] == "ok":
        assert (r.generated, r.distinct, r.depth, r.levels) == (want["generated"], want["distinct"], want["depth"],
                                                                 want["levels"])
    else:
        assert r.depth == want["depth"] and (r.generated, r.distinct) == (want["eol_generated"], want["eol_distinct"])
        assert [tlcgpu.decode(m, s) for _, s in r.trace] == [t["state"] for t in want["trace"]]
        assert ck.tlc_stop_stats() == (want["generated"], want["distinct"], want["left_on_queue"])
    ck.close()


@pytest.mark.parametrize("case", ["U_LedgerCount", "U_all_hold", "U_ContextLedgerError", "U_mixed_user_first",
                                  "U_C5_ContextBound"])
def test_user_invariant_tree_closed_mode(case):
    """the component tree's closed mode (components past a lane of the
    component engine) with the user invariants in its kernel; an error is
    replayed in TLC's order on the host (trace, TLC's stop counters)"""
    m = model(case)
    want = GOLD[case]["result"]
    ck = tlcgpu.Checker(m, engine="tree")
    r = ck.run()
    assert r.status == want["result"], (case, r.status)
    assert r.engine == "tree"
    if want["result"] == "ok":
        assert (r.generated, r.distinct, r.depth, r.levels) == (want["generated"], want["distinct"], want["depth"],
                                                                 want["levels"])
    else:
        assert r.tlc_exact and r.depth == want["depth"]
        assert (r.generated, r.distinct) == (want["eol_generated"], want["eol_distinct"])
        assert [tlcgpu.decode(m, s) for _, s in r.trace] == [t["state"] for t in want["trace"]]
        assert ck.tlc_stop_stats() == (want["generated"], want["distinct"], want["left_on_queue"])
    ck.close()


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("case", sorted(GOLD))
def test_user_invariant_ranks(case, world):
    """world 2 / 3 ranks on one GPU (tlcg_run_node): each rank's engine checks
    the user invariants on its share; the combined verdict, depth and
    end-of-level counts are the one-rank ones, and the trace walked across the
    ranks is a counterexample of the spec"""
    m = model(case)
    want = GOLD[case]["result"]
    r = tlcgpu.run_node(m, world)
    assert r.status == want["result"], (case, r.status)
    if want["result"] == "ok":
        assert (r.generated, r.distinct, r.depth, r.levels) == (want["generated"], want["distinct"], want["depth"],
                                                                 want["levels"])
        return
    assert r.depth == want["depth"]
    assert (r.generated, r.distinct) == (want["eol_generated"], want["eol_distinct"])
    if want["result"] in ("invariant", "invariant_error"):
        assert r.invariant == want["invariant"]
        check_path(m, r, want)


@pytest.mark.parametrize("case", ["U_LedgerCount", "U_all_hold", "U_ContextLedgerError", "U_producer_LedgerCount"])
def test_user_invariant_open_partition(case):
    """partition 2 (the whole state: successors cross ranks, BASELINE config
    4): the user invariants on every rank's new level, absorbed states
    included (tlcg_end_level)"""
    m = model(case)
    want = GOLD[case]["result"]
    r = tlcgpu.run_node(m, 3, partition=2, engine="global")
    assert r.status == want["result"], (case, r.status)
    assert r.depth == want["depth"]
    if want["result"] == "ok":
        assert (r.generated, r.distinct, r.levels) == (want["generated"], want["distinct"], want["levels"])
    else:
        assert (r.generated, r.distinct) == (want["eol_generated"], want["eol_distinct"])
        if want["result"] in ("invariant", "invariant_error"):
            check_path(m, r, want)


def test_user_invariant_at_scale():
    """M8 (1.1e8 states) with an invariant that holds everywhere (the
    component engine) and one that fails at depth 12 (TLC order: the global
    engine's check kernel on every level)"""
    g = GOLD["U_all_hold"]
    keys = range(1, 11)
    m = tlcgpu.Model(key_space=keys, value_space=keys, invariants=tuple(g["invariants"]), user_defs=g["user_defs"])
    r = tlcgpu.Checker(m, state_capacity=120_000_000).run(with_trace=False)
    assert (r.status, r.generated, r.distinct, r.depth) == ("ok", 147_039_563, 109_836_782, 20)
    assert r.engine == "component"
    g = GOLD["U_LedgerCount"]
    m = tlcgpu.Model(key_space=keys, value_space=keys, invariants=tuple(g["invariants"]), user_defs=g["user_defs"])
    r = tlcgpu.Checker(m, tlc_order=True, state_capacity=120_000_000).run()
    assert (r.status, r.invariant, r.depth) == ("invariant", "LedgerCount", 12)
    # the per-message-sequence law (SURVEY App.A.1): every component reaches the same depth-12 level
    assert r.distinct % tlcgpu.init_count(m) == 0


def _mutant_models():
    """semantic mutants of every fixture (user_inv_cases.semantic_mutants),
    those the product compiles, eight to a cfg's INVARIANTS list"""
    import random
    import sys
    sys.path.insert(0, HERE)
    from user_inv_cases import CASES, HELPERS, semantic_mutants
    rng = random.Random(4)
    defs, names = dict(HELPERS), []
    for name in sorted(CASES):
        for i, body in enumerate(semantic_mutants(CASES[name], rng, 8)):
            mn = f"M{len(names)}"
            trial = tlcgpu.Model(invariants=(mn,), user_defs={**HELPERS, mn: body})
            if tlcgpu.check_model(trial):
                continue  # refused (outside the supported subset)
            defs[mn] = body
            names.append(mn)
    return [tlcgpu.Model(invariants=tuple(names[i:i + 8]), user_defs=defs) for i in range(0, len(names), 8)]


@pytest.mark.parametrize("k", range(7))
def test_semantic_mutants_device_code_matches_interpreter(k, monkeypatch):
    """the generated device code in the component engine's kernel against the
    interpreter (the global engine with TLCG_JIT=0, TLC order) on semantic
    mutants of the fixtures, eight invariants a check: the same verdict,
    invariant, depth, end-of-level counts, TLC-order trace and stop counters"""
    models = _mutant_models()
    if k >= len(models):
        pytest.skip("fewer mutant groups")
    m = models[k]
    ck = tlcgpu.Checker(m)
    a = ck.run()
    stop_a = ck.tlc_stop_stats() if a.status != "ok" else None
    ck.close()
    monkeypatch.setenv("TLCG_JIT", "0")
    ck = tlcgpu.Checker(m, tlc_order=True, engine="global")
    b = ck.run()
    stop_b = ck.tlc_stop_stats() if b.status != "ok" else None
    ck.close()
    assert a.engine == "component" and b.engine == "global"
    assert (a.status, a.invariant, a.depth, a.generated, a.distinct) == \
        (b.status, b.invariant, b.depth, b.generated, b.distinct)
    if a.status != "ok":
        assert a.trace == b.trace and stop_a == stop_b
