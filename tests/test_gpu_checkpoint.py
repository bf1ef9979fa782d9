"""GPU: checkpoint / recover (TLC -checkpoint / -recover).

A run checkpointed between levels and resumed in a fresh context must end
with exactly the golden counts, per-level sizes, verdict and (TLC order)
trace of an uninterrupted run."""
import pytest

import tlcgpu
from conftest import GOLDEN, model_of
from test_gpu_parity import check_against_golden

pytestmark = pytest.mark.gpu


def run_interrupted(case, path, stop_after, tlc_order=False):
    m = model_of(GOLDEN[case]["constants"])
    a = tlcgpu.Checker(m, engine="global", tlc_order=tlc_order)
    try:
        st = a.init()
        for _ in range(stop_after):
            if st.status != 0:
                break
            st = a.step_level()
        a.checkpoint(str(path))
        before = (st.generated, st.distinct, st.depth)
    finally:
        a.close()
    b = tlcgpu.Checker(m, engine="global", tlc_order=tlc_order)
    try:
        st = b.recover(str(path))
        assert (st.generated, st.distinct, st.depth) == before
        while st.status == 0:
            st = b.step_level()
        return b.result()
    finally:
        b.close()


@pytest.mark.parametrize("case,stop_after", [("S", 7), ("S", 0), ("P_published", 5), ("W_C12_k1", 30),
                                             ("X_C5_K2", 11), ("S_consumer", 19)])
def test_resume_matches_uninterrupted(tmp_path, case, stop_after):
    r = run_interrupted(case, tmp_path / "tlcg.ckpt", stop_after)
    check_against_golden(case, r, False)


@pytest.mark.parametrize("case", ["V_leak", "V_dup_producer", "W_C12_leak"])
def test_resume_keeps_tlc_order_trace(tmp_path, case):
    r = run_interrupted(case, tmp_path / "tlcg.ckpt", 2, tlc_order=True)
    check_against_golden(case, r, True)


def test_completed_run_stays_completed(tmp_path):
    case = "S"
    m = model_of(GOLDEN[case]["constants"])
    a = tlcgpu.Checker(m, engine="global")
    a.run()
    a.checkpoint(str(tmp_path / "done.ckpt"))
    a.close()
    b = tlcgpu.Checker(m, engine="global")
    st = b.recover(str(tmp_path / "done.ckpt"))
    assert tlcgpu.STATUS[st.status] == "ok"
    check_against_golden(case, b.result(), False)
    b.close()


def test_checkpoint_refusals(tmp_path):
    m = model_of(GOLDEN["S"]["constants"])
    comp = tlcgpu.Checker(m)  # auto: the component engine finishes inside tlcg_init
    comp.init()
    with pytest.raises(RuntimeError, match="component engine"):
        comp.checkpoint(str(tmp_path / "x.ckpt"))
    comp.close()
    a = tlcgpu.Checker(m, engine="global")
    a.init()
    a.checkpoint(str(tmp_path / "s.ckpt"))
    a.close()
    other = tlcgpu.Checker(model_of(GOLDEN["S_noretain"]["constants"]), engine="global")
    with pytest.raises(RuntimeError, match="other constants"):
        other.recover(str(tmp_path / "s.ckpt"))
    with pytest.raises(RuntimeError, match="cannot read"):
        other.recover(str(tmp_path / "missing.ckpt"))
    other.close()


@pytest.mark.parametrize("damage", ["truncate", "levels", "distinct"])
def test_corrupt_checkpoint_is_refused(tmp_path, damage):
    """a truncated or corrupt checkpoint is refused with -3 before
    anything is sized from its header (no allocation from a bad count)."""
    import ctypes as C
    import struct
    path = tmp_path / "ck"
    m = model_of(GOLDEN["S"]["constants"])
    a = tlcgpu.Checker(m, engine="global")
    try:
        a.init()
        for _ in range(5):
            a.step_level()
        a.checkpoint(str(path))
    finally:
        a.close()
    raw = bytearray(path.read_bytes())
    hdr = struct.calcsize("8s8i4Q2d")
    if damage == "truncate":
        raw = raw[: len(raw) - 24]
    elif damage == "levels":  # n_levels = 2^60
        struct.pack_into("Q", raw, 8 + 32, 1 << 60)
    else:  # distinct (and the last level base) beyond the file
        struct.pack_into("Q", raw, 8 + 32 + 24, 1 << 40)
    assert hdr == 8 + 32 + 32 + 16
    path.write_bytes(bytes(raw))
    b = tlcgpu.Checker(m, engine="global")
    try:
        st = tlcgpu.tlcg_stats()
        assert b.lib.tlcg_recover(b.ctx, str(path).encode(), C.byref(st)) == -3
        assert b"corrupt" in b.lib.tlcg_last_error(b.ctx)
    finally:
        b.close()
