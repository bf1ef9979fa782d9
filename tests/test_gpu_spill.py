"""GPU: the host spill of committed levels (tlcg_opts.spill, SURVEY 8(f) row 3:
"frontier/FPSet spill to host memory for > HBM state spaces").

With a device store capped far below the state space, every level below the
frontier moves to pinned host memory; the run must still end with the golden
counts, per-level sizes, verdict and (TLC order) trace, read back the same
states, rebuild its FPSet from host memory when it grows, and checkpoint /
recover across the split."""
import pytest

import tlcgpu
from conftest import GOLDEN, model_of
from test_gpu_parity import check_against_golden
from test_gpu_partition import run_virtual

pytestmark = pytest.mark.gpu

CAP = 4096  # device store slots: a few levels of the small cases


def run_spill(case, tlc_order=False, cap=CAP, **kw):
    m = model_of(GOLDEN[case]["constants"])
    return tlcgpu.run(m, engine="global", tlc_order=tlc_order, spill=True, device_store_cap=cap, **kw)


@pytest.mark.parametrize("tlc_order", [False, True])
@pytest.mark.parametrize("case", ["S", "P_published", "W_C12_k1", "X_C5_K2", "S_consumer"])
def test_spilled_run_matches_golden(case, tlc_order):
    r = run_spill(case, tlc_order)
    check_against_golden(case, r, tlc_order)
    assert r.host_states > 0  # the levels below the frontier did leave the device
    assert r.host_states < r.distinct


@pytest.mark.parametrize("case", ["V_leak", "V_dup_producer", "W_C12_leak"])
def test_spilled_trace_is_tlcs(case):
    check_against_golden(case, run_spill(case, True, cap=256), True)


def test_spilled_store_reads_back():
    """TLC order fixes every state's index: the spilled store, read through
    tlcg_copy_states / tlcg_state_at, equals the resident one."""
    m = model_of(GOLDEN["P_published"]["constants"])
    a = tlcgpu.Checker(m, engine="global", tlc_order=True)
    b = tlcgpu.Checker(m, engine="global", tlc_order=True, spill=True, device_store_cap=CAP)
    try:
        ra, rb = a.run(), b.run()
        assert rb.host_states > 0 and (ra.distinct, ra.levels) == (rb.distinct, rb.levels)
        n = ra.distinct
        assert a.copy_states(0, n) == b.copy_states(0, n)
        # a range across the host / device split, and single states on both sides
        h = rb.host_states
        assert a.copy_states(h - 100, 200) == b.copy_states(h - 100, 200)
        for g in (0, 1, h - 1, h, n - 1):
            assert a.state_at(g) == b.state_at(g)
    finally:
        a.close()
        b.close()


def test_fpset_grows_from_host_memory():
    """An FPSet that starts at 2^16 slots grows (and is rebuilt from the
    spilled levels) several times on the way to 253361 states."""
    r = run_spill("P_published", log2_fpset_slots=0)
    check_against_golden("P_published", r, False)
    assert r.levels_redone >= 0 and r.host_states > 2 ** 16


@pytest.mark.parametrize("case,partition,world", [("P_published", 0, 3), ("S", 2, 2)])
def test_spilled_partitioned_ranks(case, partition, world):
    want = GOLDEN[case]["result"]
    gen, distinct, levels, status = run_virtual(model_of(GOLDEN[case]["constants"]), world, partition,
                                                spill=True, device_store_cap=1024)
    assert (gen, distinct, levels) == (want["generated"], want["distinct"], want["levels"])


@pytest.mark.parametrize("spill_after", [False, True])
def test_checkpoint_across_the_split(tmp_path, spill_after):
    """Checkpoint a spilled run mid-way, recover with or without spill."""
    case = "P_published"
    m = model_of(GOLDEN[case]["constants"])
    a = tlcgpu.Checker(m, engine="global", tlc_order=True, spill=True, device_store_cap=CAP)
    try:
        st = a.init()
        for _ in range(9):
            st = a.step_level()
        assert st.host_states > 0
        a.checkpoint(str(tmp_path / "c.ckpt"))
    finally:
        a.close()
    b = tlcgpu.Checker(m, engine="global", tlc_order=True, spill=spill_after, device_store_cap=CAP)
    try:
        st = b.recover(str(tmp_path / "c.ckpt"))
        assert (st.host_states > 0) == spill_after
        while st.status == 0:
            st = b.step_level()
        check_against_golden(case, b.result(), True)
    finally:
        b.close()
