"""GPU: the component-tree engine (csrc/tree.hip; Producer modelled, the
states of one `messages` value form a component and the components a tree
by prefix, compaction.tla:83-87) against the golden fixtures and the ~1e8
producer oracle run: counts, every level, depth and the generated counts
per level; the parent log it writes walks back to Init through real
successors; an error to report falls back to the global engine."""
import json
import os
import ctypes as C
import random

import pytest

import tlcgpu
from conftest import FULL_CASES, GOLDEN, model_of

pytestmark = pytest.mark.gpu

PRODUCER_CASES = [c for c in FULL_CASES if GOLDEN[c]["constants"]["producer"]]
OK_CASES = [c for c in PRODUCER_CASES if GOLDEN[c]["result"]["result"] == "ok"]
ERR_CASES = [c for c in PRODUCER_CASES if GOLDEN[c]["result"]["result"] != "ok"]


def test_there_are_producer_cases():
    assert OK_CASES and ERR_CASES


@pytest.mark.parametrize("case", OK_CASES)
def test_tree_matches_golden(case):
    m = model_of(GOLDEN[case]["constants"])
    want = GOLDEN[case]["result"]
    ck = tlcgpu.Checker(m)  # auto: the tree for <= 63-bit states, else the global engine
    try:
        r = ck.run()
        assert r.engine == ("tree" if tlcgpu.state_words(m) == 1 else "global")
        assert (r.status, r.generated, r.distinct, r.depth) == ("ok", want["generated"], want["distinct"], want["depth"])
        assert r.levels == want["levels"]
        # generated per level: the initial states, then each level's expansion, summing to the total
        g = ck.level_generated()
        assert len(g) == r.depth + 1 and sum(g) == r.generated
        # the same numbers as the global engine, level by level
        ref = tlcgpu.Checker(m, engine="global")
        try:
            ref.run()
            assert ref.level_generated() == g
        finally:
            ref.close()
    finally:
        ck.close()


@pytest.mark.parametrize("case", OK_CASES)
def test_tree_depth_counts_past_the_lds_sums(case, monkeypatch):
    """Producer mode sums the first TLCG_TREE_LVL_DEPTHS_OPEN depths' counts in
    LDS and adds deeper ones straight to the striped global counters
    (tree_body.h); with 4 LDS depths every deeper depth takes that path and the
    levels and generated counts stay the golden ones"""
    monkeypatch.setenv("TLCG_JIT", "1")
    monkeypatch.setenv("TLCG_JIT_DEFINES", "TLCG_TREE_LVL_DEPTHS_OPEN=4")
    m = model_of(GOLDEN[case]["constants"])
    if tlcgpu.state_words(m) != 1:
        pytest.skip("a wide layout: the global engine")
    want = GOLDEN[case]["result"]
    ck = tlcgpu.Checker(m)
    try:
        r = ck.run()
        assert r.engine == "tree" and r.jit_used & 1
        assert (r.status, r.generated, r.distinct, r.depth) == ("ok", want["generated"], want["distinct"], want["depth"])
        assert r.levels == want["levels"]
        g = ck.level_generated()
        assert len(g) == r.depth + 1 and sum(g) == r.generated
    finally:
        ck.close()


@pytest.mark.parametrize("case", ["P_published"])
def test_tree_parent_log_walks_to_init(case):
    """Sampled stored states (positions < 60 of random components of layers
    >= 1: every component there holds at least 62 states): each one's parent
    reference names a stored state that has it as a successor, and every chain
    ends at the initial state within the search depth."""
    c = GOLDEN[case]["constants"]
    m = model_of(c)
    nkv = (len(c["keys"]) + 1) * (len(c["values"]) + 1)
    cap = 384  # store slots per component (csrc/tree.h; these components hold <= 359 states)
    ck = tlcgpu.Checker(m, engine="tree")
    try:
        r = ck.run(with_trace=False)
        assert r.engine == "tree"
        ob = tlcgpu.load_library().tlcg_ordinal_bits(C.byref(m.to_c()))
        rng = random.Random(7)
        base, layers = cap, []  # layer 0 is one chunk
        for l in range(1, c["N"] + 1):
            layers.append((base, nkv ** l))
            base += nkv ** l * cap
        for _ in range(300):
            b0, n = rng.choice(layers)
            g = b0 + rng.randrange(n) * cap + rng.randrange(60)
            s, p = ck.state_at(g)
            steps = 0
            while p != (1 << 64) - 1:
                ps, pp = ck.state_at((p & ((1 << 56) - 1)) >> ob)
                assert s in [t for _, t in tlcgpu.host_successors(m, ps)], (case, g)
                s, p = ps, pp
                steps += 1
                assert steps < r.depth
            assert s == tlcgpu.host_init_state(m, 0)
    finally:
        ck.close()


@pytest.mark.parametrize("case", ERR_CASES)
def test_tree_error_reported_without_a_global_run(case):
    m = model_of(GOLDEN[case]["constants"])
    want = GOLDEN[case]["result"]
    ck = tlcgpu.Checker(m)  # auto: the tree finds the error and reports it (its subtree's TLC-order run)
    try:
        r = ck.run()
        assert r.engine == "tree" and r.tlc_exact
        assert r.status == want["result"] and r.depth == want["depth"]
        assert (r.generated, r.distinct) == (want["eol_generated"], want["eol_distinct"])
        if "trace" in want:
            assert [tlcgpu.decode(m, s) for _, s in r.trace] == [t["state"] for t in want["trace"]]
            assert ck.tlc_stop_stats() == (want["generated"], want["distinct"], want["left_on_queue"])
        # the next check on the same context runs the tree again (fast order)
        r2 = ck.run()
        assert (r2.status, r2.generated, r2.distinct) == (r.status, r.generated, r.distinct)
    finally:
        ck.close()


@pytest.mark.parametrize("jit", ["0", "1"])
@pytest.mark.parametrize("case", ["W_C12_leak", "W_C12_dup"])
def test_tree_closed_error_reported(case, jit, monkeypatch):
    """the tree's closed mode (wide components) finds TLC's first error: its
    least error key names the component, which the host replays in TLC order
    (verdict, depth, end-of-level counts, trace); TLCG_JIT=1 runs the wave
    kernel (tree_wave.h), whose violators come from one evaluation per flag
    combination (a ballot) and whose keys are folded per lane"""
    monkeypatch.setenv("TLCG_JIT", jit)
    m = model_of(GOLDEN[case]["constants"])
    want = GOLDEN[case]["result"]
    ck = tlcgpu.Checker(m)
    try:
        r = ck.run()
        assert r.engine == "tree" and bool(r.jit_used & 16) == (jit == "1")
        assert r.status == want["result"] and r.depth == want["depth"]
        assert (r.generated, r.distinct) == (want["eol_generated"], want["eol_distinct"])
        if "trace" in want:
            assert [tlcgpu.decode(m, s) for _, s in r.trace] == [t["state"] for t in want["trace"]]
    finally:
        ck.close()


def test_p8_on_the_tree():
    """~1e8 producer-modelled states (tests/golden/p8.json, from the C oracle)."""
    g = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "p8.json")))
    ck = tlcgpu.Checker(model_of(g["constants"]), engine="tree")
    try:
        r = ck.run()
        want = g["result"]
        assert r.engine == "tree"
        assert (r.generated, r.distinct, r.depth) == (want["generated"], want["distinct"], want["depth"])
        assert r.levels == want["levels"]
        # a second check on the same context gives the same numbers
        r2 = ck.run()
        assert (r2.generated, r2.distinct, r2.levels) == (r.generated, r.distinct, r.levels)
    finally:
        ck.close()


INVARIANTS = ["TypeSafe", "CompactedLedgerLeak", "CompactionHorizonCorrectness", "DuplicateNullKeyMessage"]


def random_producer_model(seed):
    """A seeded producer-modelled constant set (every other knob drawn too),
    small enough for the C oracle to finish in well under a second."""
    rng = random.Random(1000 + seed)
    return tlcgpu.Model(msg_sent_limit=rng.randint(1, 3), compaction_times_limit=rng.choice([1, 2, 3, 4]),
                        max_crash_times=rng.randint(0, 2), consume_times_limit=rng.randint(0, 2),
                        model_consumer=rng.random() < 0.3, model_producer=True,
                        retain_null_key=rng.random() < 0.6,
                        key_space=sorted(rng.sample(range(1, 9), rng.randint(0, 2))),
                        value_space=sorted(rng.sample(range(1, 9), rng.randint(0, 2))),
                        invariants=rng.sample(INVARIANTS, rng.randint(1, 4)), check_deadlock=rng.random() < 0.5)


def tree_applies(m):
    """the tree keeps 31-bit local keys: the state above `messages` and its
    length (csrc/model.h layout; tree_applicable in csrc/tlcgpu.hip)"""
    n = m.msg_sent_limit
    kb = len(m.key_space).bit_length()    # key indices 0..|KeySpace| (0 = NullKey)
    vb = len(m.value_space).bit_length()
    mb = n.bit_length() + n * (kb + vb)
    return tlcgpu.state_words(m) == 1 and tlcgpu.state_bits(m) - mb <= 31


@pytest.mark.parametrize("seed", range(60))
def test_tree_random_producer_cfgs(seed):
    """Seeded random producer-modelled cfgs against the C oracle run live: the
    tree's counts and every level when the check passes; on an error the
    verdict, the depth, the end-of-level counts, TLC's trace and TLC's stop
    counters, reported by the tree (its erroring subtree run in TLC order) or
    by the global engine in TLC order (an error of the root component or at
    level 1, or a model the tree does not take)."""
    from conftest import run_oracle
    m = random_producer_model(seed)
    if tlcgpu.check_model(m) is not None:
        pytest.skip(f"constants refused: {tlcgpu.check_model(m)}")
    want = run_oracle(m)
    ck = tlcgpu.Checker(m)
    r = ck.run()
    stop = ck.tlc_stop_stats() if r.status != "ok" else None
    ck.close()
    assert r.status == want["result"], (seed, r.status, want["result"])
    assert r.depth == want["depth"], seed
    if want["result"] == "ok":
        assert (r.generated, r.distinct, r.levels) == (want["generated"], want["distinct"], want["levels"]), seed
        assert r.engine == ("tree" if tree_applies(m) else "global"), (seed, r.engine)
    else:
        assert r.engine in ("tree", "global") and r.tlc_exact, (seed, r.engine)
        if want["result"] in ("invariant", "invariant_error"):
            assert r.invariant == want["invariant"], seed
        assert (r.generated, r.distinct) == (want["eol_generated"], want["eol_distinct"]), seed
        assert [tlcgpu.decode(m, s) for _, s in r.trace] == [t["state"] for t in want["trace"]], seed
        assert stop == (want["generated"], want["distinct"], want["left_on_queue"]), (seed, r.engine)


@pytest.mark.parametrize("ranks", [2, 3, 8])
def test_tree_sharded_over_ranks(ranks):
    """with the Producer modelled, `ranks` contexts (tlcg_run_node,
    threads on this one GPU) each run whole subtrees of the component tree --
    the layer that first has >= `ranks` components is split into contiguous
    ranges, the layers above it run everywhere and count once -- with no
    exchange; the combined counts and every level are the golden ones"""
    for case in OK_CASES:
        m = model_of(GOLDEN[case]["constants"])
        if tlcgpu.state_words(m) != 1:
            continue
        want = GOLDEN[case]["result"]
        r = tlcgpu.run_node(m, ranks)
        assert r.engine == "tree", case
        assert (r.status, r.generated, r.distinct, r.depth) == ("ok", want["generated"], want["distinct"],
                                                                 want["depth"]), case
        assert r.levels == want["levels"], case
    g = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "p8.json")))
    r = tlcgpu.run_node(model_of(g["constants"]), ranks)
    want = g["result"]
    assert r.engine == "tree"
    assert (r.generated, r.distinct, r.depth, r.levels) == (want["generated"], want["distinct"], want["depth"],
                                                             want["levels"])


@pytest.mark.parametrize("seed", range(10))
def test_tree_sharded_random_producer_cfgs(seed):
    """seeded random producer cfgs at 2 and 5 ranks against the C oracle run
    live: counts and levels when the check passes; on an error the ranks hand
    the model to the global engine's exchange, which reports TLC's verdict"""
    from conftest import run_oracle
    m = random_producer_model(seed)
    if tlcgpu.check_model(m) is not None:
        pytest.skip(f"constants refused: {tlcgpu.check_model(m)}")
    want = run_oracle(m)
    for ranks in (2, 5):
        r = tlcgpu.run_node(m, ranks)
        assert r.status == want["result"], (seed, ranks, r.status)
        assert r.depth == want["depth"], (seed, ranks)
        if want["result"] == "ok":
            assert (r.generated, r.distinct, r.levels) == (want["generated"], want["distinct"], want["levels"])
            assert r.engine == ("tree" if tree_applies(m) else "global"), (seed, r.engine)
        else:
            assert r.engine == "global"
            assert (r.generated, r.distinct) == (want["eol_generated"], want["eol_distinct"]), (seed, ranks)


@pytest.mark.parametrize("case", ERR_CASES)
def test_tree_sharded_error_hands_over_to_the_exchange(case):
    m = model_of(GOLDEN[case]["constants"])
    want = GOLDEN[case]["result"]
    r = tlcgpu.run_node(m, 3)
    assert r.engine == "global"
    assert r.status == want["result"] and r.depth == want["depth"]
    assert (r.generated, r.distinct) == (want["eol_generated"], want["eol_distinct"])


@pytest.mark.parametrize("jit", ["0", "1"])
def test_tree_closed_store_reads_back_states(jit, monkeypatch):
    """the closed mode stores component codes (tree_body.h TLCG_TREE_CODE_STORE);
    tlcg_copy_states / tlcg_state_at decode them: the first component's chunk
    holds exactly its reachable states, each one's parent reference names a
    state of the chunk that has it as a successor.  TLCG_JIT=1: the hipRTC
    kernels, whose first pass walks each code graph once per wavefront
    (tree_wave.h) into a lane-interleaved store: component 0's position i is
    slot 64 i (tree_wave_slot)"""
    monkeypatch.setenv("TLCG_JIT", jit)
    c = GOLDEN["W_C12_k1"]["constants"]
    m = model_of(c)
    ck = tlcgpu.Checker(m)
    try:
        r = ck.run()
        assert r.engine == "tree"
        wave = bool(r.jit_used & 16)
        assert wave == (jit == "1")
        step = 64 if wave else 1  # slot of component 0's next position
        s0 = tlcgpu.host_init_state(m, 0)
        seen, todo = set(), [s0]
        while todo:
            s = todo.pop()
            if s not in seen:
                seen.add(s)
                todo += [t for _, t in tlcgpu.host_successors(m, s)]
        n = len(seen)
        assert n == r.distinct // tlcgpu.init_count(m)
        stored = ck.copy_states(0, n * step)[::step]
        assert set(stored) == seen and stored[0] == s0
        ob = tlcgpu.load_library().tlcg_ordinal_bits(C.byref(m.to_c()))
        for i in range(1, n, 7):
            s, p = ck.state_at(i * step)
            assert s == stored[i]
            pg = (p & ((1 << 56) - 1)) >> ob
            assert pg % step == 0
            ps, _ = ck.state_at(pg)
            assert s in [t for _, t in tlcgpu.host_successors(m, ps)]
    finally:
        ck.close()


@pytest.mark.parametrize("jit", ["0", "1"])
def test_tree_closed_store_last_component(jit, monkeypatch):
    """W_C12 has 729 components, so the wave kernel's last row of
    64 is padded (25 components, 39 empty lanes).  The whole last row copies
    back (padded lanes read as 'no walk'), and the last component's slots hold
    exactly its reachable states, its initial state first; TLCG_JIT=0: the
    chunk layout (component ci at ci x 640)"""
    monkeypatch.setenv("TLCG_JIT", jit)
    m = model_of(GOLDEN["W_C12"]["constants"])
    nc = tlcgpu.init_count(m)
    assert nc % 64 != 0
    cap = 640  # closed mode's store slots per component (csrc/tree.h, tlcg_treec_640)
    ck = tlcgpu.Checker(m)
    try:
        r = ck.run()
        assert r.engine == "tree"
        wave = bool(r.jit_used & 16)
        assert wave == (jit == "1")
        ci = nc - 1
        s0 = tlcgpu.host_init_state(m, ci)
        seen, todo = set(), [s0]
        while todo:
            s = todo.pop()
            if s not in seen:
                seen.add(s)
                todo += [t for _, t in tlcgpu.host_successors(m, s)]
        n = len(seen)
        assert n * nc == r.distinct
        if wave:
            row = ck.copy_states(ci // 64 * 64 * cap, 64 * cap)  # the last row, padded lanes included
            stored = row[ci % 64::64][:n]
        else:
            stored = ck.copy_states(ci * cap, n)
        assert set(stored) == seen and stored[0] == s0
    finally:
        ck.close()


@pytest.mark.parametrize("case,mode", [("P_published", "auto"), ("W_C12", "perlane"), ("W_C12", "wave")])
def test_tree_expansions_count(case, mode, monkeypatch):
    """tlcg_expansions on the component tree: each component's states are
    expanded once at their depth (tree_body.h; the Producer tree and the closed
    mode's per-state passes), so distinct / expansions = 1; the closed mode's
    wave kernel (tree_wave.h) expands each walk's code states once for all its
    components (W_C12: 557 code states per walk, 729 components)"""
    if mode == "perlane":
        monkeypatch.setenv("TLCG_JIT", "1")
        monkeypatch.setenv("TLCG_TREE_WAVE", "0")
    elif mode == "wave":
        monkeypatch.setenv("TLCG_JIT", "1")
    m = model_of(GOLDEN[case]["constants"])
    ck = tlcgpu.Checker(m)
    try:
        r = ck.run(with_trace=False)
        assert r.engine == "tree" and r.distinct == GOLDEN[case]["result"]["distinct"]
        x = ck.expansions()
        if mode == "wave":
            assert r.jit_used & 16
            n = r.distinct // tlcgpu.init_count(m)
            assert x % n == 0 and 0 < x < r.distinct, (x, n)
        else:
            assert x == r.distinct, (x, r.distinct)
    finally:
        ck.close()
