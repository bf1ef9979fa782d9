"""The component tree's closed-mode slot hash, replayed on the host (no GPU).

Without a Producer every component of a model has the same code graph, so
the engine builds a perfect-hash displacement table from component 0's code
set (build_slot_disp, host_model.cpp) and the kernel's inserts take one CAS
each (tree_body.h).  These tests check that claim on components other than
the one the table was built from, through tlcg_host_tree_slot_probes: with
the table every insert call's longest lane probes once; without it, linear
probing at the 640-slot table's load takes more.  Counts are not at stake
here (linear probing stays behind the table; the GPU parity tests pin them);
this pins the property the G9-deep timing rests on."""
import pytest

import tlcgpu


def model(keys, C, retain=True):
    return tlcgpu.Model(key_space=range(1, keys + 1), value_space=range(1, keys + 1),
                        compaction_times_limit=C, retain_null_key=retain)


@pytest.mark.parametrize("keys,C", [(10, 12), (3, 12), (4, 9), (2, 10)])
def test_perfect_hash_on_every_sampled_component(keys, C):
    m = model(keys, C)
    n = tlcgpu.init_count(m)
    for comp in sorted({0, 1, 2, n // 3, n // 2, n - 2, n - 1}):
        r = tlcgpu.host_tree_slot_probes(m, comp)
        assert r is not None, comp
        calls, trips, plain = r
        assert calls > 0
        assert trips == calls, (comp, r)  # one CAS per insert
        assert plain >= calls


def test_g9deep_linear_probing_alone_takes_longer():
    # BASELINE's G9-deep: 557 states per component in 640 slots
    calls, trips, plain = tlcgpu.host_tree_slot_probes(model(10, 12), 12345)
    assert trips == calls
    assert plain > 3 * calls  # (3.76 per call with the tuned multiplier alone)


def test_not_taken_with_a_producer():
    m = tlcgpu.Model(model_producer=True)
    assert tlcgpu.host_tree_slot_probes(m, 0) is None
