"""GPU: the HIP checker (libtlcgpu.so on an MI355X) against the golden
fixtures made by the CPU oracle -- counts, per-level sizes, depth, verdict,
and the counterexample trace text (TLC-order mode) -- plus size-independent
checks at the ~1e8 / ~1e9 scaled configs."""
import random

import pytest

import tlcgpu
from conftest import FULL_CASES, GOLDEN, model_of

pytestmark = pytest.mark.gpu

G9 = dict(key_space=range(1, 16), value_space=range(1, 16))
M8 = dict(key_space=range(1, 11), value_space=range(1, 11))


def check_against_golden(case, r, tlc_order):
    want = GOLDEN[case]["result"]
    assert r.status == want["result"], (case, r.status)
    if want["result"] == "ok":
        assert (r.generated, r.distinct, r.depth) == (want["generated"], want["distinct"], want["depth"])
        assert r.levels == want["levels"]
        assert r.left_on_queue == 0
        return
    # an error stops the run at the end of the level that found it: the depth
    # and the trace are TLC's; generated/distinct are counted to that level end
    # (the oracles' eol_* counts), the same for every engine and order
    assert r.depth == want["depth"], (case, r.engine, r.depth)
    assert (r.generated, r.distinct) == (want["eol_generated"], want["eol_distinct"]), (case, r.engine)
    assert sum(r.levels) == r.distinct, (case, r.engine)
    m = model_of(GOLDEN[case]["constants"])
    want_trace = want["trace"]
    assert len(r.trace) == len(want_trace)
    if want["result"] == "invariant":
        assert r.invariant == want["invariant"]
    if tlc_order or r.engine == "component" or r.tlc_exact:  # each reproduces TLC's -workers 1 trace
        assert [a for a, _ in r.trace] == [t["action"] for t in want_trace]
        assert [tlcgpu.decode(m, s) for _, s in r.trace] == [t["state"] for t in want_trace]
    else:
        # any shortest counterexample: a valid path from an initial state
        assert r.trace[0][0] == "Init"
        for (_, s), (a, t) in zip(r.trace, r.trace[1:]):
            assert (a, t) in tlcgpu.host_successors(m, s)
        if want["result"] == "invariant":
            c = tlcgpu.host_check_invariants(m, r.trace[-1][1])
            assert c >= 0 and m.invariants[c >> 1] == want["invariant"]


@pytest.mark.parametrize("mode", ["auto", "global", "tlc_order"])
@pytest.mark.parametrize("case", FULL_CASES)
def test_golden_case(case, mode):
    m = model_of(GOLDEN[case]["constants"])
    r = tlcgpu.run(m, tlc_order=mode == "tlc_order", engine="global" if mode == "global" else "auto")
    check_against_golden(case, r, mode == "tlc_order")
    c = GOLDEN[case]["constants"]
    if mode == "auto" and not c["producer"] and want_ok(case):
        # components are isomorphic (SURVEY App.A.1): all fit on chip iff one does
        g = GOLDEN[case]["result"]
        per_component = g["distinct"] // tlcgpu.init_count(m)
        fits = per_component <= 255 and g["depth"] <= 47 and component_key_fits(c)
        # a component too large for a lane goes to the component tree's closed
        # mode when its codes fit (csrc/tree.h), else to the global engine
        tree = code_bits(c) <= 31 and per_component <= 2048 and g["depth"] <= 126
        assert r.engine == ("component" if fits else "tree" if tree else "global"), (r.engine, per_component)


ERROR_CASES = [c for c in FULL_CASES if GOLDEN[c]["result"]["result"] != "ok"]


@pytest.mark.parametrize("store", ["resident", "spilled"])
@pytest.mark.parametrize("case", ERROR_CASES)
def test_tlc_stop_statistics(case, store):
    """TLC's "G states generated, D distinct states found, Q states left on
    queue." where a one-worker run stops on the error (tlcg_tlc_stop_stats):
    the oracles' stop point, with the levels in HBM or mostly spilled to host
    memory (a 256-state device store)."""
    m = model_of(GOLDEN[case]["constants"])
    want = GOLDEN[case]["result"]
    kw = dict(spill=True, device_store_cap=256) if store == "spilled" else {}
    ck = tlcgpu.Checker(m, tlc_order=True, engine="global", **kw)
    try:
        r = ck.run()
        assert r.status == want["result"]
        assert ck.tlc_stop_stats() == (want["generated"], want["distinct"], want["left_on_queue"]), case
    finally:
        ck.close()


OK_CASES = [c for c in FULL_CASES if GOLDEN[c]["result"]["result"] == "ok"]


@pytest.mark.parametrize("mode", ["auto", "tlc_order"])
@pytest.mark.parametrize("case", OK_CASES)
def test_outdegree_histogram(case, mode):
    """TLC's outdegree statistics (new states discovered per expanded state,
    over TLC's first-discoverer tree) against both oracles' histogram: from the
    component engine's lanes, or from the runs of equal parent in every sorted
    TLC-order level.  The global engine in fast order refuses (its parents are
    whichever insert won)."""
    m = model_of(GOLDEN[case]["constants"])
    ck = tlcgpu.Checker(m, tlc_order=mode == "tlc_order", engine="global" if mode == "tlc_order" else "auto",
                        outdegree=True)
    try:
        r = ck.run()
        assert r.status == "ok"
        if mode == "tlc_order" or r.engine == "component":
            assert ck.outdegree() == GOLDEN[case]["result"]["outdegree"], (case, mode, r.engine)
        else:
            with pytest.raises(RuntimeError):
                ck.outdegree()
    finally:
        ck.close()


def test_tlc_stop_statistics_need_tlc_order():
    """The global engine outside TLC order: its store is not in TLC's FIFO
    order, so its stop statistics are refused (the on-chip engines give them,
    test_tlc_stop_statistics_without_a_rerun)."""
    m = model_of(GOLDEN["V_leak"]["constants"])
    ck = tlcgpu.Checker(m, engine="global")
    try:
        r = ck.run()
        assert r.status == "invariant" and not r.tlc_exact
        with pytest.raises(RuntimeError):
            ck.tlc_stop_stats()
    finally:
        ck.close()


@pytest.mark.parametrize("case", ERROR_CASES)
def test_tlc_stop_statistics_without_a_rerun(case):
    """the default engine reports TLC's first error itself.
    Closed partitions: the component engine (TLC-order lanes) or the component
    tree's closed mode (the error's component replayed in TLC's order on the
    host) -- trace and TLC's stop counters with no global-engine run (the
    components before the error's counted by a prefix run of the same
    engine).  Producer modelled: the tree's error switches the one-rank run to
    the global engine in TLC order, so its trace and counters need no second
    run either."""
    m = model_of(GOLDEN[case]["constants"])
    want = GOLDEN[case]["result"]
    ck = tlcgpu.Checker(m)
    try:
        r = ck.run()
        assert r.status == want["result"]
        if r.engine == "global" and not m.model_producer:
            pytest.skip("no on-chip engine takes this model")
        assert r.tlc_exact, (case, r.engine)
        if m.model_producer:
            assert r.engine in ("tree", "global")
        assert [a for a, _ in r.trace] == [t["action"] for t in want["trace"]], (case, r.engine)
        assert [tlcgpu.decode(m, s) for _, s in r.trace] == [t["state"] for t in want["trace"]]
        assert (r.generated, r.distinct) == (want["eol_generated"], want["eol_distinct"])
        assert ck.tlc_stop_stats() == (want["generated"], want["distinct"], want["left_on_queue"]), (case, r.engine)
        # the same context checks again
        r2 = ck.run()
        assert (r2.status, r2.generated, r2.distinct, r2.engine) == (r.status, r.generated, r.distinct, r.engine)
    finally:
        ck.close()


def component_key_fits(c):
    """the component engine's admission rule: a one-word state whose part above
    `messages` (the local key) fits 32 bits (tlcgpu.hip component_applicable)"""
    m = model_of(c)
    nk, nv = len(set(c["keys"]) | {0}), len(set(c["values"]) | {0})
    led_sh = c["N"].bit_length() + c["N"] * ((nk - 1).bit_length() + (nv - 1).bit_length())
    bits = tlcgpu.state_bits(m)
    return bits <= 63 and bits - led_sh <= 32 and c["N"] <= 8


def code_bits(c):
    """bits of a component code (csrc/component_code.h): C presence bits, 5
    (readPosition, horizon, phase), context and cursor context, 2 (cursor
    present, cursor horizon), crash count"""
    return c["C"] + 7 + 2 * c["C"].bit_length() + c["K"].bit_length()


def want_ok(case):
    return GOLDEN[case]["result"]["result"] == "ok"


def per_m_law(case_first_m, n_m, r):
    one = GOLDEN[case_first_m]["result"]
    assert r.status == "ok"
    assert r.distinct == n_m * one["distinct"]
    # generated: one initial state per M is counted once per M
    assert r.generated == n_m * one["generated"]
    assert r.depth == one["depth"]
    assert r.levels == [n_m * x for x in one["levels"]]


def test_m8_scaled_counts():
    # ~1e8: KeySpace = ValueSpace = 1..10 -> 11^6 message sequences x 62
    r = tlcgpu.run(tlcgpu.Model(**M8))
    per_m_law("M8_first_M", 11 ** 6, r)
    assert r.distinct == 109_836_782 and r.generated == 147_039_563


def test_g9_scaled_counts_and_parent_log():
    # ~1e9: KeySpace = ValueSpace = 1..15 -> 16^6 message sequences x 62
    m = tlcgpu.Model(**G9)
    ck = tlcgpu.Checker(m, log2_fpset_slots=31, state_capacity=1_100_000_000, engine="global")
    try:
        r = ck.run(with_trace=False)
        per_m_law("G9_first_M", 16 ** 6, r)
        assert r.distinct == 1_040_187_392 and r.generated == 1_392_508_928
        # parent-pointer log: every sampled state is its parent's successor at the
        # recorded Next ordinal, and the parent sits one level up
        bounds = [0]
        for x in r.levels:
            bounds.append(bounds[-1] + x)
        rng = random.Random(7)
        lib = tlcgpu.load_library()
        ordbits = lib.tlcg_ordinal_bits(__import__("ctypes").byref(m.to_c()))
        for _ in range(300):
            g = rng.randrange(bounds[1], r.distinct)
            s, pref = ck.state_at(g)
            pg, ordinal = (pref & ((1 << 56) - 1)) >> ordbits, pref & ((1 << ordbits) - 1)
            lvl = next(i for i in range(len(bounds) - 1) if bounds[i] <= g < bounds[i + 1])
            assert bounds[lvl - 1] <= pg < bounds[lvl]
            ps, _ = ck.state_at(pg)
            act = tlcgpu.ACTIONS[lib.tlcg_action_of_ordinal(__import__("ctypes").byref(m.to_c()), ordinal)]
            assert (act, s) in tlcgpu.host_successors(m, ps)
        # the stored levels are duplicate-free
        sample = ck.copy_states(bounds[5], min(2_000_000, r.levels[5]))
        assert len(set(sample)) == len(sample)
    finally:
        ck.close()


def test_growth_and_redo_paths():
    # a 2^10-slot FPSet and a tiny store force FPSet/store growth and level redo
    m = model_of(GOLDEN["P_published"]["constants"])
    ck = tlcgpu.Checker(m, log2_fpset_slots=10, state_capacity=1000, engine="global")
    try:
        r = ck.run()
        check_against_golden("P_published", r, False)
        assert r.levels_redone > 0
    finally:
        ck.close()


def test_rerun_same_context_is_identical():
    m = model_of(GOLDEN["S"]["constants"])
    ck = tlcgpu.Checker(m, tlc_order=True)
    try:
        a = ck.run()
        sa = ck.copy_states(0, a.distinct)
        b = ck.run()
        sb = ck.copy_states(0, b.distinct)
        assert (a.generated, a.distinct, a.levels) == (b.generated, b.distinct, b.levels)
        assert sa == sb  # TLC-order mode: the store order is deterministic
    finally:
        ck.close()


def test_tlc_order_levels_are_sorted_by_discovery():
    m = model_of(GOLDEN["X_producer_sparse"]["constants"])
    ck = tlcgpu.Checker(m, tlc_order=True)
    try:
        r = ck.run()
        lib = tlcgpu.load_library()
        import ctypes
        ordbits = lib.tlcg_ordinal_bits(ctypes.byref(m.to_c()))
        refs = [ck.state_at(g)[1] for g in range(r.levels[0], r.distinct)]
        start = r.levels[0]
        for n in r.levels[1:]:
            lvl = refs[:n]
            refs = refs[n:]
            assert lvl == sorted(lvl)
            start += n
        assert ordbits > 0
    finally:
        ck.close()


def test_g9_component_engine():
    # the component engine on the ~1e9 config: same counts and per-level sizes
    m = tlcgpu.Model(**G9)
    ck = tlcgpu.Checker(m, engine="component")
    try:
        r = ck.run(with_trace=False)
        assert r.engine == "component"
        per_m_law("G9_first_M", 16 ** 6, r)
        # spot-check the store: component 0 (lane 0 of batch 0) is message sequence M0,
        # stored FIFO at gidx 64 * position; parents point one level up the chain
        s0, p0 = ck.state_at(0)
        assert s0 == tlcgpu.host_init_state(m, 0) and p0 == (1 << 64) - 1
        s1, p1 = ck.state_at(64)
        assert ("CompactorPhaseOne", s1) in tlcgpu.host_successors(m, s0)
    finally:
        ck.close()


def test_g9_component_wave_records_decode():
    """G9 on the component engine's wave kernel (csrc/component_wave.h): the
    records are the walks' (one per walk and queue position), and every
    component's slot still decodes (tlcgpu.hip crec_index, comp_slot_decode):
    sampled components read back their initial state at position 0, and every
    sampled state is a successor of its recorded parent (same lane, an earlier
    position) by the recorded action"""
    import ctypes
    m = tlcgpu.Model(**G9)
    ck = tlcgpu.Checker(m)
    try:
        r = ck.run(with_trace=False)
        assert r.engine == "component" and r.jit_used & 8
        assert r.distinct == 1_040_187_392
        lib = tlcgpu.load_library()
        ob = lib.tlcg_ordinal_bits(ctypes.byref(m.to_c()))
        rng = random.Random(11)
        for _ in range(200):
            ci = rng.randrange(16 ** 6)
            row = (ci // 64) * 64 * 64 + ci % 64  # (K = 64: slot = batch x 4096 + position x 64 + lane)
            s0, p0 = ck.state_at(row)
            assert s0 == tlcgpu.host_init_state(m, ci) and p0 == (1 << 64) - 1  # (NO_PARENT)
            g = row + 64 * rng.randrange(1, 62)  # every G9 component holds 62 states
            s, pref = ck.state_at(g)
            pg, ordinal = (pref & ((1 << 56) - 1)) >> ob, pref & ((1 << ob) - 1)
            assert pg % 64 == ci % 64 and row <= pg < g
            ps, _ = ck.state_at(pg)
            act = tlcgpu.ACTIONS[lib.tlcg_action_of_ordinal(ctypes.byref(m.to_c()), ordinal)]
            assert (act, s) in tlcgpu.host_successors(m, ps)
    finally:
        ck.close()


@pytest.mark.parametrize("case", ["X_keys3_vals57", "S_consumer", "S_noretain", "R_C3_K1"])
@pytest.mark.parametrize("jit", ["0", "1"])
def test_component_code_records_decode(jit, case, monkeypatch):
    """The code pass stores one 32-bit record per state (csrc/component.h
    comp_record: code, parent queue position, action) and tlcg_state_at /
    tlcg_copy_states rebuild the state word and the parent reference from the
    slot: component ci (lane ci % 64 of batch ci // 64) reads back, at
    positions 0..n-1, exactly its n reachable states in BFS order, position 0
    its initial state without a parent, every other state a successor of an
    earlier position of the same lane by the recorded action.  Precompiled
    (TLCG_JIT=0) and hipRTC-specialized (1) kernels."""
    monkeypatch.setenv("TLCG_JIT", jit)
    m = model_of(GOLDEN[case]["constants"])
    ck = tlcgpu.Checker(m, engine="component")
    try:
        r = ck.run(with_trace=False)
        assert r.engine == "component"
        check_against_golden(case, r, False)
        lib = tlcgpu.load_library()
        import ctypes
        ob = lib.tlcg_ordinal_bits(ctypes.byref(m.to_c()))
        n_init = tlcgpu.init_count(m)
        checked = 0
        for ci in sorted(set(range(0, min(n_init, 130))) | {n_init - 1}):
            seen, order = {tlcgpu.host_init_state(m, ci)}, [tlcgpu.host_init_state(m, ci)]
            for s in order:  # the component's closure (no Producer: `messages` is fixed)
                for _, t in tlcgpu.host_successors(m, s):
                    if t not in seen:
                        seen.add(t)
                        order.append(t)
            if len(order) > 62:  # (K - 1 or more states: the cascade's word store)
                continue
            base = (ci // 64) * 64 * 64 + ci % 64
            slots = [base + 64 * p for p in range(len(order))]
            got = ck.copy_states(slots[0], slots[-1] - slots[0] + 1)[::64]
            assert set(got) == seen and got[0] == order[0]
            for p, g in enumerate(slots):
                s, pref = ck.state_at(g)
                assert s == got[p]
                if p == 0:
                    assert pref == (1 << 64) - 1
                    continue
                pg, ordinal = (pref & ((1 << 56) - 1)) >> ob, pref & ((1 << ob) - 1)
                assert pg in slots[:p]
                ps, _ = ck.state_at(pg)
                act = tlcgpu.ACTIONS[lib.tlcg_action_of_ordinal(ctypes.byref(m.to_c()), ordinal)]
                assert (act, s) in tlcgpu.host_successors(m, ps)
            checked += 1
        assert checked >= min(100, n_init)
    finally:
        ck.close()


def test_component_engine_multi_rank_ranges():
    m = model_of(GOLDEN["X_keys3_vals57"]["constants"])
    want = GOLDEN["X_keys3_vals57"]["result"]
    tot_g = tot_d = 0
    for rank in range(3):
        ck = tlcgpu.Checker(m, rank=rank, world=3, engine="component")
        try:
            r = ck.run(with_trace=False)
            tot_g += r.generated
            tot_d += r.distinct
        finally:
            ck.close()
    assert (tot_g, tot_d) == (want["generated"], want["distinct"])


@pytest.mark.parametrize("case", ["S", "R_C4_K1", "R_C5_K1", "R_C4_K3", "V_leak", "V_dup", "X_keys3_vals57",
                                  "D_N0_K1", "S_consumer"])
def test_component_cascade(case, monkeypatch):
    # start the on-chip cascade at 32 states per component: components of
    # 33..255 states overflow and are redone at 64/128/255; levels counted before
    # the overflow are not counted twice
    monkeypatch.setenv("TLCG_COMP_K0", "32")
    m = model_of(GOLDEN[case]["constants"])
    r = tlcgpu.run(m)
    check_against_golden(case, r, False)


@pytest.mark.parametrize("engine", ["auto", "global"])
def test_g9deep_scaled_counts(engine):
    """KeySpace = ValueSpace = 1..10, CompactionTimesLimit
    = 12 -> a 93-bit state (two words): 11^6 x 557 = 986,759,477 distinct,
    1,119,626,552 generated, depth 74 -- on the component tree's closed mode
    (auto: 557-state components on 28-bit codes) and on the wide FPSet."""
    m = tlcgpu.Model(compaction_times_limit=12, **M8)
    assert tlcgpu.state_words(m) == 2
    kw = dict(log2_fpset_slots=31, state_capacity=1_000_000_000) if engine == "global" else {}
    r = tlcgpu.run(m, engine=engine, **kw)
    per_m_law("G9deep_first_M", 11 ** 6, r)
    assert (r.distinct, r.generated, r.depth) == (986_759_477, 1_119_626_552, 74)
    assert r.engine == ("tree" if engine == "auto" else "global")



@pytest.mark.parametrize("engine", ["auto", "global"])
def test_p8_producer_scaled_matches_oracle(engine):
    """An open (producer-modelled) state space of ~1e8 states on the
    component-tree engine (auto) and on the global engine: KeySpace =
    ValueSpace = 1..7, ModelProducer, RetainNullKey FALSE; counts and every
    level against the C oracle (tests/golden/p8.json)."""
    import json
    import os
    g = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "p8.json")))
    r = tlcgpu.run(model_of(g["constants"]), engine=engine)
    want = g["result"]
    assert r.engine == ("tree" if engine == "auto" else "global") and r.status == "ok"
    assert (r.generated, r.distinct, r.depth, r.levels) == (want["generated"], want["distinct"], want["depth"],
                                                            want["levels"])
