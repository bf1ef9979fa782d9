"""GPU: every first-pass kernel of the on-chip engines against the golden
fixtures and the live oracle, error paths included.

The default engine picks its kernel by size: the hipRTC-specialized kernels
from 65,536 components on, and among them the one-walk-per-wavefront kernels
(component_wave.h, tree_wave.h) with the big-model variant (16 components per
lane) from 2^23 components on.  The golden cases are small, so here each
kernel is forced on them:

  wave        TLCG_JIT=1: tlcg_componentw_64 (M = 10) / tlcg_treecw_640
  wave_big    + TLCG_WAVE_BIG_COMPS=1: the big-model module (M = 16)
  perlane     TLCG_JIT=1, TLCG_COMP_WAVE=0, TLCG_TREE_WAVE=0: the per-lane kernels,
              bench.py's per-state headline -- tlcg_componentp_64 (component_lane.h,
              a bitmap FPSet) where its slot hash exists, else tlcg_componentc_64
              (component_body.h) / tlcg_treec_640
  perlane_body  the same with TLCG_COMP_LANE=0 and TLCG_TREE_BITS=0: tlcg_componentc_64
              and the closed tree's code tables (tlcg_treec_640) throughout
  refuse_odd  TLCG_JIT=1 and the test hook TLCG_WAVE_REFUSE_ODD: the components
              of odd batch + lane parity refuse the walk, so the walk-join
              fallback (component_wave.h) and the 32-bit cascade pass run

and the counts, levels, verdict, depth, TLC-order trace and TLC's stop
counters must be the oracle's."""
import random

import pytest

import tlcgpu
from conftest import FULL_CASES, GOLDEN, model_of, run_oracle
from test_gpu_parity import check_against_golden
from test_gpu_random_cfgs import random_model

pytestmark = pytest.mark.gpu

MODES = {
    "wave": {"TLCG_JIT": "1"},
    "wave_big": {"TLCG_JIT": "1", "TLCG_WAVE_BIG_COMPS": "1"},
    "perlane": {"TLCG_JIT": "1", "TLCG_COMP_WAVE": "0", "TLCG_TREE_WAVE": "0"},
    "perlane_body": {"TLCG_JIT": "1", "TLCG_COMP_WAVE": "0", "TLCG_TREE_WAVE": "0", "TLCG_COMP_LANE": "0",
                     "TLCG_TREE_BITS": "0"},
    "refuse_odd": {"TLCG_JIT": "1", "TLCG_JIT_DEFINES": "TLCG_WAVE_REFUSE_ODD=1"},
}


def set_mode(monkeypatch, mode):
    for k, v in MODES[mode].items():
        monkeypatch.setenv(k, v)


def check_kernel(mode, r):
    """the forced kernel is the one that ran (when an on-chip engine took the model)"""
    if r.engine == "component" and r.jit_used & 2:  # (the code pass)
        assert r.jit_used & 1, r.jit_used
        assert bool(r.jit_used & 8) == (not mode.startswith("perlane")), (mode, r.jit_used)
        if mode == "perlane_body":
            assert not r.jit_used & 32, r.jit_used
    if r.engine == "tree" and mode.startswith("perlane"):
        assert not r.jit_used & 16, r.jit_used
        if mode == "perlane_body":
            assert not r.jit_used & 128, r.jit_used


@pytest.mark.parametrize("mode", sorted(MODES))
@pytest.mark.parametrize("case", FULL_CASES)
def test_golden_case_kernel(case, mode, monkeypatch):
    set_mode(monkeypatch, mode)
    m = model_of(GOLDEN[case]["constants"])
    r = tlcgpu.run(m)
    check_against_golden(case, r, False)
    check_kernel(mode, r)


ERROR_CASES = [c for c in FULL_CASES if GOLDEN[c]["result"]["result"] != "ok"]


@pytest.mark.parametrize("mode", sorted(MODES))
@pytest.mark.parametrize("case", ERROR_CASES)
def test_tlc_stop_statistics_kernel(case, mode, monkeypatch):
    """the default engine's error report with each kernel: TLC's trace, the
    end-of-level counts and TLC's stop counters, without a global re-run"""
    set_mode(monkeypatch, mode)
    m = model_of(GOLDEN[case]["constants"])
    want = GOLDEN[case]["result"]
    ck = tlcgpu.Checker(m)
    try:
        r = ck.run()
        assert r.status == want["result"]
        check_kernel(mode, r)
        if r.engine == "global" and not m.model_producer:
            pytest.skip("no on-chip engine takes this model")
        assert r.tlc_exact, (case, r.engine)
        assert [a for a, _ in r.trace] == [t["action"] for t in want["trace"]], (case, r.engine)
        assert [tlcgpu.decode(m, s) for _, s in r.trace] == [t["state"] for t in want["trace"]]
        assert (r.generated, r.distinct) == (want["eol_generated"], want["eol_distinct"])
        assert ck.tlc_stop_stats() == (want["generated"], want["distinct"], want["left_on_queue"]), (case, r.engine)
    finally:
        ck.close()


@pytest.mark.parametrize("mode", ["perlane", "refuse_odd"])
@pytest.mark.parametrize("seed", range(40))
def test_random_cfg_kernel(seed, mode, monkeypatch):
    """tests/test_gpu_random_cfgs.py's seeded constants on the default engine
    with each kernel, against the oracle run live"""
    m = random_model(seed)
    if tlcgpu.check_model(m) is not None:
        pytest.skip(f"constants refused: {tlcgpu.check_model(m)}")
    set_mode(monkeypatch, mode)
    want = run_oracle(m)
    ck = tlcgpu.Checker(m, outdegree=mode.startswith("perlane"))
    try:
        r = ck.run()
        check_kernel(mode, r)
        assert r.status == want["result"], (seed, mode, r.status, want["result"])
        if want["result"] == "ok":
            assert (r.generated, r.distinct, r.depth, r.levels) == \
                   (want["generated"], want["distinct"], want["depth"], want["levels"]), (seed, mode)
            if mode.startswith("perlane") and r.engine == "component":  # TLC's first-discoverer tree
                assert ck.outdegree() == want["outdegree"], (seed, mode)
            return
        assert r.depth == want["depth"], (seed, mode)
        if want["result"] in ("invariant", "invariant_error"):
            assert r.invariant == want["invariant"], (seed, mode)
        if r.tlc_exact:
            assert [tlcgpu.decode(m, s) for _, s in r.trace] == [t["state"] for t in want["trace"]], (seed, mode)
            assert (r.generated, r.distinct) == (want["eol_generated"], want["eol_distinct"]), (seed, mode)
            assert ck.tlc_stop_stats() == (want["generated"], want["distinct"], want["left_on_queue"]), seed
    finally:
        ck.close()


G9 = dict(key_space=range(1, 16), value_space=range(1, 16))


@pytest.mark.parametrize("case", ["S", "V_leak", "V_dup", "S_noretain", "X_keys3_vals57", "R_C2_K2"])
def test_lane_pass_runs(case, monkeypatch):
    """the per-lane bitmap pass (component_lane.h, jit_used bit 5) is the
    per-state kernel wherever its slot hash exists (components of <= 62
    states): here, with the golden result"""
    set_mode(monkeypatch, "perlane")
    m = model_of(GOLDEN[case]["constants"])
    r = tlcgpu.run(m)
    check_against_golden(case, r, False)
    assert r.engine == "component" and r.jit_used & 32 and not r.jit_used & 8, r.jit_used


@pytest.mark.parametrize("ring", ["4", "16"])
@pytest.mark.parametrize("case", ["S", "V_leak", "V_dup", "R_C2_K2"])
def test_lane_ring_size(case, ring, monkeypatch):
    """the per-lane pass's FIFO ring (component_lane.h LANE_R) is sized per
    layout by the host (host_model.cpp lane_ring_entries: 8 when component 0's
    widest queue fits); forced to 4, components whose queue outgrows it leave
    the pass for the cascade (the `full` branch), and to 16 the pre-sizing
    ring: both with the golden result, error reports included"""
    set_mode(monkeypatch, "perlane")
    monkeypatch.setenv("TLCG_JIT_DEFINES", "TLCG_LANE_R=" + ring)
    m = model_of(GOLDEN[case]["constants"])
    r = tlcgpu.run(m)
    check_against_golden(case, r, False)
    assert r.engine == "component" and r.jit_used & 32, r.jit_used


def test_g9_lane_ring_4_cascades_exactly(monkeypatch):
    """G9 with a 4-entry ring: every component outgrows it and the 32-bit
    cascade redoes it, counting only the levels the lane pass left open"""
    set_mode(monkeypatch, "perlane")
    monkeypatch.setenv("TLCG_JIT_DEFINES", "TLCG_LANE_R=4")
    m = tlcgpu.Model(**G9)
    ck = tlcgpu.Checker(m)
    try:
        r = ck.run(with_trace=False)
        assert r.engine == "component" and r.jit_used & 32
        assert (r.distinct, r.generated, r.depth) == (1_040_187_392, 1_392_508_928, 20)
    finally:
        ck.close()


@pytest.mark.parametrize("mode", ["default", "perlane", "perlane_body"])
def test_g9_ledger_leak(mode, monkeypatch):
    """G9 (16^6 components, so the default engine runs the big-model wave
    variant) with CompactedLedgerLeak (compaction.tla:253) in the cfg: every
    component violates it at depth 12.  TLC's first error is component 0's
    (the least initial state), so the trace is the oracle's on component 0
    alone, and the counts at the end of the error's level follow the per-M law
    (every component has the same code graph): 16^6 x the oracle's one-
    component end-of-level counts.  The law itself is checked on the oracle's
    first 4,096 components."""
    if mode != "default":
        set_mode(monkeypatch, mode)
    m = tlcgpu.Model(invariants=("TypeSafe", "CompactedLedgerLeak", "CompactionHorizonCorrectness"), **G9)
    one = run_oracle(m, ["-init-lo", "0", "-init-hi", "1"])
    many = run_oracle(m, ["-init-lo", "0", "-init-hi", "4096", "-notrace"])
    assert one["result"] == many["result"] == "invariant" and one["depth"] == many["depth"] == 12
    assert (many["eol_generated"], many["eol_distinct"]) == (4096 * one["eol_generated"], 4096 * one["eol_distinct"])
    n = 16 ** 6
    ck = tlcgpu.Checker(m)
    try:
        r = ck.run()
        assert r.engine == "component"
        assert bool(r.jit_used & 8) == (mode == "default"), r.jit_used
        assert bool(r.jit_used & 32) == (mode == "perlane"), r.jit_used  # (component_lane.h's bitmap pass)
        assert (r.status, r.invariant, r.depth) == ("invariant", "CompactedLedgerLeak", 12)
        assert r.tlc_exact
        assert [a for a, _ in r.trace] == [t["action"] for t in one["trace"]]
        assert [tlcgpu.decode(m, s) for _, s in r.trace] == [t["state"] for t in one["trace"]]
        assert (r.generated, r.distinct) == (n * one["eol_generated"], n * one["eol_distinct"])
        # (the oracle's levels stop at the violating state; the last one is cut there)
        assert len(r.levels) == 12 and sum(r.levels) == r.distinct
        assert r.levels[:-1] == [n * x for x in one["levels"][:-1]]
    finally:
        ck.close()


@pytest.mark.parametrize("defines", ["", "TLCG_WAVE_M=7"])
def test_g9_wave_module_m_override(defines, monkeypatch):
    """the wave module's components per lane come from the
    module (tlcg_wave_m, jit.cpp), and the host's grid and record tables
    (crec_index) follow it -- built with M = 7 by a define (the big variant's
    16 otherwise), G9's counts are exact and sampled components read back
    their states through their walk's records"""
    import ctypes
    if defines:
        monkeypatch.setenv("TLCG_JIT_DEFINES", defines)
    m = tlcgpu.Model(**G9)
    ck = tlcgpu.Checker(m)
    try:
        r = ck.run(with_trace=False)
        assert r.engine == "component" and r.jit_used & 8
        assert (r.distinct, r.generated) == (1_040_187_392, 1_392_508_928)
        lib = tlcgpu.load_library()
        ob = lib.tlcg_ordinal_bits(ctypes.byref(m.to_c()))
        rng = random.Random(13)
        for ci in [0, 63, 64, 7 * 64 - 1, 7 * 64, 16 ** 6 - 1] + [rng.randrange(16 ** 6) for _ in range(150)]:
            row = (ci // 64) * 64 * 64 + ci % 64  # (K = 64: slot = batch x 4096 + position x 64 + lane)
            s0, p0 = ck.state_at(row)
            assert s0 == tlcgpu.host_init_state(m, ci) and p0 == (1 << 64) - 1
            g = row + 64 * rng.randrange(1, 62)
            s, pref = ck.state_at(g)
            pg, ordinal = (pref & ((1 << 56) - 1)) >> ob, pref & ((1 << ob) - 1)
            assert pg % 64 == ci % 64 and row <= pg < g
            ps, _ = ck.state_at(pg)
            act = tlcgpu.ACTIONS[lib.tlcg_action_of_ordinal(ctypes.byref(m.to_c()), ordinal)]
            assert (act, s) in tlcgpu.host_successors(m, ps)
        # a whole component's 62 slots through tlcg_copy_states (crec_index over a walk's row)
        ci = 7 * 64 + 5
        row = (ci // 64) * 64 * 64 + ci % 64
        got = ck.copy_states(row, 61 * 64 + 1)[::64]
        seen, order = {tlcgpu.host_init_state(m, ci)}, [tlcgpu.host_init_state(m, ci)]
        for s in order:
            for _, t in tlcgpu.host_successors(m, s):
                if t not in seen:
                    seen.add(t)
                    order.append(t)
        assert got == order
    finally:
        ck.close()


@pytest.mark.parametrize("mode", ["perlane", "perlane_body", "wave", "global"])
def test_expansions_count(mode, monkeypatch):
    """tlcg_expansions, the kernels' own count of state expansions: a per-lane
    kernel expands every distinct state once (distinct / expansions = 1), the
    one-walk-per-wavefront kernel each code state of a walk once for all its
    components (M8: ceil(11^6 / 64 / M) walks x 62 code states), the global
    engine each stored level once"""
    m = tlcgpu.Model(key_space=range(1, 11), value_space=range(1, 11))
    if mode != "global":
        set_mode(monkeypatch, mode)
    ck = tlcgpu.Checker(m, engine="global" if mode == "global" else "auto",
                        log2_fpset_slots=28 if mode == "global" else 0)
    try:
        r = ck.run(with_trace=False)
        assert (r.distinct, r.generated) == (109_836_782, 147_039_563)
        x = ck.expansions()
        if mode == "wave":
            assert r.jit_used & 8
            walks = -(-(-(-11 ** 6 // 64)) // 10)  # (M = 10: M8 is under WAVE_BIG_COMPS)
            assert x == walks * 62, (x, walks)
        else:
            assert x == r.distinct, (mode, x, r.distinct)
    finally:
        ck.close()


@pytest.mark.parametrize("case", FULL_CASES)
def test_golden_case_global_specialized(case, monkeypatch):
    """the global engine's fast level built layout-specialized (expand_fast.h
    through jit.cpp, tlcg_stats.jit_used bit 6), forced onto the golden cases
    with TLCG_JIT=1: the golden result (one-word layouts without a Producer
    take the fast level; the others keep their kernels)"""
    monkeypatch.setenv("TLCG_JIT", "1")
    m = model_of(GOLDEN[case]["constants"])
    r = tlcgpu.run(m, engine="global")
    check_against_golden(case, r, False)
    if tlcgpu.state_words(m) == 1 and not m.model_producer:
        assert r.jit_used & 64, r.jit_used


@pytest.mark.parametrize("groups", ["", "TLCG_TREECB_G=4"])
@pytest.mark.parametrize("case", ["W_C12", "W_C12_k1", "W_C12_noretain", "W_C12_leak", "W_C12_dup"])
def test_tree_bits_pass_runs(case, groups, monkeypatch):
    """the closed tree's per-state pass with the bitmap FPSet (tree_body.h
    BITS, jit_used bit 7) takes the wide golden cases when its perfect hash
    exists: the golden result, at its 16 components per wavefront (tree.h
    TREECB_G) and at 4 (the module's define; the host's grid stays sized for
    16, and the kernel strides over the rest)"""
    set_mode(monkeypatch, "perlane")
    if groups:
        monkeypatch.setenv("TLCG_JIT_DEFINES", groups)
    m = model_of(GOLDEN[case]["constants"])
    r = tlcgpu.run(m)
    check_against_golden(case, r, False)
    assert r.engine == "tree" and r.jit_used & 128 and not r.jit_used & 16, r.jit_used
