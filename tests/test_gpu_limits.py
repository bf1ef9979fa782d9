"""GPU: the largest constants this build takes, pinned by the scaling laws of
SURVEY App.A.3 (R(C,1) = 3C^2 + 10C + 5 distinct states for one message
sequence, depth 6C + 2; distinct = (|KeySet||ValueSet|)^N * R) and, where it
reaches, by the CPU oracle."""
import json
import subprocess

import pytest

import tlcgpu
from conftest import ORACLE

pytestmark = pytest.mark.gpu


def r_c1(C):
    return 3 * C * C + 10 * C + 5


@pytest.mark.parametrize("C", [12, 13, 14, 16, 24, 32])
def test_compaction_times_limit_up_to_32(C):
    """CompactionTimesLimit up to the build's maximum (32): one initial state
    (KeySpace = ValueSpace = {}, N = 1); C >= 24 are wide (two-word) layouts.
    C = 12 / 13 / 14 put the one component at 557 / 642 / 733 states, around
    the component tree's 640-state chunk: 642 fills the chunk's table within
    its last depth, which must send the component on to the 2048-state pass
    (ADVICE r2), not drop states."""
    m = tlcgpu.Model(msg_sent_limit=1, compaction_times_limit=C, key_space=[], value_space=[])
    r = tlcgpu.run(m)
    assert r.status == "ok"
    assert (r.distinct, r.depth) == (r_c1(C), 6 * C + 2)
    if C <= 16:  # the C oracle's range
        want = json.loads(subprocess.run([ORACLE] + m.oracle_args() + ["-levels"], check=True,
                                         capture_output=True, text=True).stdout)
        assert (r.generated, r.distinct, r.depth, r.levels) == (want["generated"], want["distinct"],
                                                                want["depth"], want["levels"])


def test_compaction_times_limit_33_is_refused():
    m = tlcgpu.Model(msg_sent_limit=1, compaction_times_limit=33, key_space=[], value_space=[])
    assert "CompactionTimesLimit > 32" in tlcgpu.check_model(m)


def test_largest_key_space():
    """|KeySpace| = 63, the ABI maximum (tlcgpu.h TLCG_MAX_SET): 64 keys (NullKey
    included) x 2 values, 128^3 message sequences x R(3,1) = 62 states each."""
    m = tlcgpu.Model(key_space=range(1, 64), value_space=[1])
    r = tlcgpu.run(m)
    assert r.status == "ok"
    assert r.distinct == 128 ** 3 * 62 and r.generated == 128 ** 3 * 83 and r.depth == 20
    with pytest.raises(ValueError):
        tlcgpu.Model(key_space=range(1, 65)).to_c()
