"""GPU: the host FPSet tier (tlcg_opts.fpset_spill, SURVEY 8(f) row 3, TLC's
DiskFPSet).

With the HBM table capped at 2^12 slots (2^10 for the traces), every few levels its states move to a
sorted run in host memory behind an HBM Bloom filter, and each level's new
states are checked against the runs.  Counts, per-level sizes, verdicts and
TLC-order traces must equal the golden ones."""
import pytest

import tlcgpu
from conftest import GOLDEN, model_of
from test_gpu_parity import check_against_golden
from test_gpu_partition import run_virtual

pytestmark = pytest.mark.gpu

TIER = dict(engine="global", fpset_spill=True, log2_fpset_max=12)


def tiered(case, tlc_order=False, **kw):
    m = model_of(GOLDEN[case]["constants"])
    return tlcgpu.run(m, tlc_order=tlc_order, **TIER, **kw)


@pytest.mark.parametrize("tlc_order", [False, True])
@pytest.mark.parametrize("case", ["S", "P_published", "S_consumer", "S_noretain", "X_keys3_vals57"])
def test_tiered_run_matches_golden(case, tlc_order):
    r = tiered(case, tlc_order)
    check_against_golden(case, r, tlc_order)
    # more states than a 2^12-slot table holds at load 1/2: the host tier took some
    assert r.fpset_host_states > 0


@pytest.mark.parametrize("case", ["V_leak", "V_dup_producer"])
def test_tiered_trace_is_tlcs(case):
    m = model_of(GOLDEN[case]["constants"])
    r = tlcgpu.run(m, tlc_order=True, **dict(TIER, log2_fpset_max=10))
    check_against_golden(case, r, True)
    assert r.fpset_host_states > 0


def test_tier_with_store_spill():
    """Both host tiers at once: the store window and the FPSet runs."""
    r = tiered("P_published", True, spill=True, device_store_cap=4096)
    check_against_golden("P_published", r, True)
    assert r.fpset_host_states > 0 and r.host_states > 0


@pytest.mark.parametrize("case,partition,world", [("P_published", 0, 3), ("S", 2, 2)])
def test_tiered_partitioned_ranks(case, partition, world):
    want = GOLDEN[case]["result"]
    gen, distinct, levels, status = run_virtual(model_of(GOLDEN[case]["constants"]), world, partition,
                                                fpset_spill=True, log2_fpset_max=12)
    assert (gen, distinct, levels) == (want["generated"], want["distinct"], want["levels"])


def test_recover_into_the_tier(tmp_path):
    """A checkpoint too large for the capped table recovers into host runs."""
    case = "P_published"
    m = model_of(GOLDEN[case]["constants"])
    a = tlcgpu.Checker(m, engine="global", tlc_order=True)
    try:
        st = a.init()
        for _ in range(14):
            st = a.step_level()
        assert st.distinct > 2 ** 12
        a.checkpoint(str(tmp_path / "c.ckpt"))
    finally:
        a.close()
    b = tlcgpu.Checker(m, tlc_order=True, **TIER)
    try:
        st = b.recover(str(tmp_path / "c.ckpt"))
        assert st.fpset_host_states > 0
        while st.status == 0:
            st = b.step_level()
        check_against_golden(case, b.result(), True)
    finally:
        b.close()


def test_tier_refuses_wide_states():
    m = model_of(GOLDEN["W_C12_k1"]["constants"])
    assert tlcgpu.state_words(m) == 2
    with pytest.raises(RuntimeError, match="63-bit"):
        tlcgpu.Checker(m, **TIER)
