"""GPU: the fingerprint-partitioned FPSet (tlcg_expand/outbox/inbox/absorb/
end_level) with W virtual ranks as W contexts on one MI355X, the all-to-all
done by device copies.  Counts must not depend on W (multi-GPU
without a cluster)."""
import pytest
import torch

import dist as tdist
import tlcgpu
from conftest import GOLDEN, model_of

pytestmark = pytest.mark.gpu


def run_virtual(model, world, partition=0, **opts):
    # (the exchange API itself: an open partition runs the global engine, not
    # the component tree's sharded subtrees that tlcg_init would otherwise run)
    if model.model_producer or partition == 2:
        opts.setdefault("engine", "global")
    engines = [tdist.GpuEngine(model, r, world, 0, partition=partition, **opts) for r in range(world)]
    try:
        if engines[0].closed:
            stats = [e.run_closed() for e in engines]
            gen = sum(s.generated for s in stats)
            distinct = sum(s.distinct for s in stats)
            levels = {}
            for e in engines:
                for i, x in enumerate(e.level_sizes()):
                    levels[i] = levels.get(i, 0) + x
            lv = [levels[i] for i in sorted(levels)]
            while lv and lv[-1] == 0:
                lv.pop()
            return gen, distinct, lv, max(s.status for s in stats)
        stats = [e.init() for e in engines]
        while True:
            if any(s.status >= 2 for s in stats) or sum(e.level_sizes()[-1] for e in engines) == 0:
                break
            for e in engines:
                e.expand()
            for dst in range(world):
                parts = [engines[src].outbox(dst) for src in range(world) if src != dst]
                recs = torch.cat(parts, 0) if parts else torch.empty((0, 2), dtype=torch.int64, device="cuda:0")
                if recs.shape[0]:
                    engines[dst].absorb(recs)
            stats = [e.end_level() for e in engines]
        gen = sum(s.generated for s in stats)
        distinct = sum(s.distinct for s in stats)
        lv = [sum(x) for x in zip(*[e.level_sizes() for e in engines])]
        while lv and lv[-1] == 0:
            lv.pop()
        # open partition: the ranks stay "running"; the driver ends the run
        st = max(s.status for s in stats)
        return gen, distinct, lv, st if st >= 2 else 1
    finally:
        for e in engines:
            e.close()


@pytest.mark.parametrize("world", [2, 3, 8])
@pytest.mark.parametrize("case,partition", [("S", 0), ("S", 2), ("P_published", 0), ("X_producer_sparse", 0),
                                            ("X_keys3_vals57", 2)])
def test_partition_counts_invariant_in_world(case, partition, world):
    want = GOLDEN[case]["result"]
    gen, distinct, levels, status = run_virtual(model_of(GOLDEN[case]["constants"]), world, partition)
    assert status == 1
    assert (gen, distinct, levels) == (want["generated"], want["distinct"], want["levels"])


def test_partition_owner_is_a_function_of_messages_when_closed():
    m = tlcgpu.Model()
    e = tdist.GpuEngine(m, 0, 4, 0)
    try:
        lib = tlcgpu.load_library()
        s = tlcgpu.host_init_state(m, 77)
        owners = {lib.tlcg_owner(e.ctx, t) for _, t in tlcgpu.host_successors(m, s)}
        owners.add(lib.tlcg_owner(e.ctx, s))
        assert len(owners) == 1 and e.closed
    finally:
        e.close()


def test_m8_partitioned_matches_single():
    m = tlcgpu.Model(key_space=range(1, 11), value_space=range(1, 11))
    gen, distinct, levels, status = run_virtual(m, 4)
    assert (gen, distinct, status) == (147_039_563, 109_836_782, 1)
    assert len(levels) == 20


# ---- tlcg_run_node: one process drives every rank (tlc-hip -gpus N) ----

@pytest.mark.parametrize("ranks", [2, 3, 8])
@pytest.mark.parametrize("case,partition", [("S", 0), ("S", 2), ("P_published", 0), ("X_producer_sparse", 0),
                                            ("X_keys3_vals57", 2), ("W_C12", 0), ("D_N0_K1", 0)])
def test_run_node_counts_invariant_in_ranks(case, partition, ranks):
    want = GOLDEN[case]["result"]
    r = tlcgpu.run_node(model_of(GOLDEN[case]["constants"]), ranks, partition=partition)
    assert r.status == want["result"]
    assert (r.generated, r.distinct, r.depth, r.levels) == (want["generated"], want["distinct"], want["depth"],
                                                             want["levels"])


@pytest.mark.parametrize("ranks", [2, 4])
@pytest.mark.parametrize("case,partition", [("V_leak", 0), ("V_dup", 0), ("V_leak_producer", 0), ("V_leak", 2)])
def test_run_node_violation_verdict(case, partition, ranks):
    want = GOLDEN[case]["result"]
    r = tlcgpu.run_node(model_of(GOLDEN[case]["constants"]), ranks, partition=partition)
    assert (r.status, r.invariant, r.depth) == (want["result"], want["invariant"], want["depth"])


@pytest.mark.parametrize("pipeline", ["1", "0"])
@pytest.mark.parametrize("case", ["S", "V_leak"])
def test_run_node_pipelined_level_overflows(case, pipeline, monkeypatch):
    """the one-wait level (csrc/tlcgpu.hip ctx_absorb_expand: absorb, end of
    level and next expand on the stream back to back) and the two-step level
    (TLCG_PIPELINE=0) report the same counts and verdict when the outboxes
    start at 64 records per destination (TLCG_OUTBOX_CAP) and overflow, so
    the expand's redo paths run, from tiny store and FPSet sizes"""
    monkeypatch.setenv("TLCG_PIPELINE", pipeline)
    monkeypatch.setenv("TLCG_OUTBOX_CAP", "64")  # the first outbox of each buffer overflows
    want = GOLDEN[case]["result"]
    r = tlcgpu.run_node(model_of(GOLDEN[case]["constants"]), 3, partition=2, engine="global", log2_fpset_slots=8,
                        state_capacity=256)
    assert r.status == want["result"]
    if want["result"] == "ok":
        assert (r.generated, r.distinct, r.depth, r.levels) == (want["generated"], want["distinct"], want["depth"],
                                                                 want["levels"])
    else:
        assert (r.invariant, r.depth) == (want["invariant"], want["depth"])
        assert (r.generated, r.distinct) == (want["eol_generated"], want["eol_distinct"])
    assert r.levels_redone > 0


def test_run_node_matches_checker_engines():
    # the closed partition runs either engine per rank; the open one the global engine
    m = model_of(GOLDEN["S"]["constants"])
    want = GOLDEN["S"]["result"]
    for engine in ("auto", "global", "component"):
        r = tlcgpu.run_node(m, 4, engine=engine)
        assert (r.generated, r.distinct, r.levels) == (want["generated"], want["distinct"], want["levels"])


@pytest.mark.parametrize("ranks", [2, 4])
@pytest.mark.parametrize("case,partition", [("V_leak", 0), ("V_dup", 0), ("V_leak_producer", 0), ("V_leak", 2)])
def test_run_node_error_counts_at_level_end(case, partition, ranks):
    """every rank's counts cut at the end of the first error's level: the
    counts one context reports (the oracles' eol_* numbers)"""
    want = GOLDEN[case]["result"]
    r = tlcgpu.run_node(model_of(GOLDEN[case]["constants"]), ranks, partition=partition)
    assert (r.generated, r.distinct) == (want["eol_generated"], want["eol_distinct"])
    assert r.levels[:-1] == want["levels"][:-1] and sum(r.levels) == r.distinct
    assert r.transport == "local"  # ranks share the one GPU


def check_behavior(m, want, trace):
    """a shortest behavior of the spec ending in the golden case's error: an
    initial state, one Next step per state (host_successors, the model.h
    semantics the oracles pin), as long as TLC's trace, its last state
    violating the reported invariant (or without a successor: deadlock)"""
    assert len(trace) == len(want["trace"])
    assert trace[0][0] == "Init"
    assert trace[0][1] in {tlcgpu.host_init_state(m, i) for i in range(tlcgpu.init_count(m))}
    for (_, s), (a, t) in zip(trace, trace[1:]):
        assert (a, t) in tlcgpu.host_successors(m, s)
    last = trace[-1][1]
    if want["result"] == "invariant":
        code = tlcgpu.host_check_invariants(m, last)
        assert code >= 0 and m.invariants[code >> 1] == want["invariant"]
        # and no shorter prefix violates
        assert all(tlcgpu.host_check_invariants(m, s) < 0 for _, s in trace[:-1])
    else:
        assert want["result"] == "deadlock" and not tlcgpu.host_successors(m, last)


@pytest.mark.parametrize("ranks", [2, 4, 8])
@pytest.mark.parametrize("case,partition", [("V_leak", 0), ("V_dup", 0), ("V_leak_producer", 0), ("V_dup_producer", 0),
                                            ("V_leak", 2), ("V_dup", 2), ("D_N0_K1", 0), ("D_N0_K1", 2),
                                            ("W_C12_leak", 0)])
def test_run_node_trace_across_ranks(case, partition, ranks):
    """the first error's counterexample walked across the ranks'
    stores without a re-run (tlcg_run_node_trace; csrc/tlcgpu.hip
    trace_ranks): with partition 2 and with the Producer the chain crosses
    ranks, state by state, through the parent references that name them"""
    want = GOLDEN[case]["result"]
    m = model_of(GOLDEN[case]["constants"])
    r = tlcgpu.run_node(m, ranks, partition=partition)
    assert (r.status, r.depth) == (want["result"], want["depth"])
    check_behavior(m, want, r.trace)


def test_run_node_trace_empty_when_the_model_holds():
    r = tlcgpu.run_node(model_of(GOLDEN["S"]["constants"]), 4, partition=2)
    assert r.status == "ok" and r.trace == []


@pytest.mark.parametrize("case", ["V_leak", "V_dup_producer"])
def test_run_comm_trace_world1(case):
    """tlcg_run_comm over the RCCL transport (world 1) leaves the walked
    counterexample for tlcg_trace_words"""
    import ctypes as C
    want = GOLDEN[case]["result"]
    m = model_of(GOLDEN[case]["constants"])
    ck = tlcgpu.Checker(m)
    try:
        lib = ck.lib
        buf = C.create_string_buffer(128)
        assert lib.tlcg_comm_unique_id(buf, 128) == 128
        assert lib.tlcg_comm_init(ck.ctx, buf, 128) == 0, lib.tlcg_last_error(ck.ctx)
        st = tlcgpu.tlcg_stats()
        assert lib.tlcg_run_comm(ck.ctx, C.byref(st), None, 0, None) == 0, lib.tlcg_last_error(ck.ctx)
        assert tlcgpu.STATUS[st.status] == want["result"]
        check_behavior(m, want, ck.trace())
    finally:
        ck.close()


# SURVEY App.A.2: distinct states per BFS level of one initial message sequence
PER_M_LEVELS = [1, 2, 2, 3, 3, 3, 4, 3, 3, 4, 4, 3, 4, 4, 4, 5, 5, 1, 2, 2]


def test_g9_hash_partitioned_8_ranks():
    """BASELINE config 4 on one GPU: G9 (~1e9 states) with the FPSet
    partitioned on the whole state (owner = mix64(state), partition 2) over 8
    ranks, so every BFS level runs expand -> all-to-all of records -> absorb
    (tlcg_run_node, the level loop of tlcg_run_comm with the local transport).
    Exact counts, depth and per-level sizes."""
    m = tlcgpu.Model(key_space=range(1, 16), value_space=range(1, 16))
    per = 1_040_187_392 // 8 + 1
    r = tlcgpu.run_node(m, 8, partition=2, engine="global", log2_fpset_slots=(2 * per - 1).bit_length(),
                        state_capacity=int(per * 1.1) + (1 << 20))
    assert (r.status, r.generated, r.distinct, r.depth) == ("ok", 1_392_508_928, 1_040_187_392, 20)
    assert r.levels == [16 ** 6 * x for x in PER_M_LEVELS]
    assert r.transport == "local"
    # owner and FPSet slot come from independent hash bits: each rank's table at
    # load 1/2 never overflows, so no level is redone
    assert r.levels_redone == 0


@pytest.mark.parametrize("case,partition", [("S", 0), ("P_published", 0), ("V_leak", 0), ("V_leak_producer", 0)])
def test_run_node_rccl_transport(case, partition, monkeypatch):
    """the RCCL transport (ncclCommInitAll, all-reduces of the combine) with
    one rank on the one GPU of the box; the driver's 8-GPU node runs it with
    records moving over xGMI"""
    monkeypatch.setenv("TLCG_NODE_TRANSPORT", "rccl")
    want = GOLDEN[case]["result"]
    r = tlcgpu.run_node(model_of(GOLDEN[case]["constants"]), 1, partition=partition)
    assert r.transport == "rccl"
    assert r.status == want["result"]
    if want["result"] == "ok":
        assert (r.generated, r.distinct, r.depth, r.levels) == (want["generated"], want["distinct"], want["depth"],
                                                                 want["levels"])
    else:
        assert (r.generated, r.distinct, r.depth) == (want["eol_generated"], want["eol_distinct"], want["depth"])


def test_native_comm_world1():
    """tlcg_comm_unique_id -> tlcg_comm_init -> tlcg_run_comm (what
    dist.run_native drives per process), twice on one communicator"""
    import ctypes as C
    m = model_of(GOLDEN["P_published"]["constants"])
    want = GOLDEN["P_published"]["result"]
    ck = tlcgpu.Checker(m)
    try:
        lib = ck.lib
        assert lib.tlcg_comm_available() == 1
        buf = C.create_string_buffer(128)
        assert lib.tlcg_comm_unique_id(buf, 128) == 128
        assert lib.tlcg_comm_init(ck.ctx, buf, 128) == 0, lib.tlcg_last_error(ck.ctx)
        for _ in range(2):
            st = tlcgpu.tlcg_stats()
            lv = (C.c_uint64 * 4096)()
            n = C.c_int32()
            assert lib.tlcg_run_comm(ck.ctx, C.byref(st), lv, 4096, C.byref(n)) == 0, lib.tlcg_last_error(ck.ctx)
            assert (st.generated, st.distinct, st.depth, st.transport) == (want["generated"], want["distinct"],
                                                                           want["depth"], 2)
            assert [lv[i] for i in range(n.value)] == want["levels"]
    finally:
        ck.close()


def test_run_comm_without_communicator_is_refused():
    import ctypes as C
    ck = tlcgpu.Checker(tlcgpu.Model())
    try:
        st = tlcgpu.tlcg_stats()
        assert ck.lib.tlcg_run_comm(ck.ctx, C.byref(st), None, 0, None) < 0
        assert b"no communicator" in ck.lib.tlcg_last_error(ck.ctx)
    finally:
        ck.close()
