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


def test_run_node_matches_checker_engines():
    # the closed partition runs either engine per rank; the open one the global engine
    m = model_of(GOLDEN["S"]["constants"])
    want = GOLDEN["S"]["result"]
    for engine in ("auto", "global", "component"):
        r = tlcgpu.run_node(m, 4, engine=engine)
        assert (r.generated, r.distinct, r.levels) == (want["generated"], want["distinct"], want["levels"])
