"""GPU: seeded random constant sets, beyond the golden fixtures, against the C
oracle run live on the same inputs (oracle/build/tlc_oracle, the checker).
Counts, per-level sizes, depth and verdict through the default engine and the
global engine in TLC order; on an error, TLC's trace text and TLC's
statistics at the stop (tlcg_tlc_stop_stats); on success, TLC's outdegree
histogram (tlcg_outdegree).

The draws cover every knob of compaction.cfg: MessageSentLimit 0..3,
CompactionTimesLimit 1..6 (wide > 63-bit layouts included), MaxCrashTimes
0..2, sparse KeySpace/ValueSpace (empty included), RetainNullKey, the
Producer and Consumer switches, ConsumeTimesLimit, CHECK_DEADLOCK and any
ordered subset of the four invariants (compaction.tla:236-294)."""
import random

import pytest

import tlcgpu
from conftest import run_oracle

pytestmark = pytest.mark.gpu

INVARIANTS = ["TypeSafe", "CompactedLedgerLeak", "CompactionHorizonCorrectness", "DuplicateNullKeyMessage"]


def random_model(seed):
    rng = random.Random(seed)
    producer = rng.random() < 0.35
    # keep every draw to <= a few 1e5 states so the oracle finishes in well under a second
    small = 2 if producer else 3
    keys = sorted(rng.sample(range(1, 9), rng.randint(0, small)))
    values = sorted(rng.sample(range(1, 9), rng.randint(0, small)))
    return tlcgpu.Model(msg_sent_limit=rng.randint(0, 3),
                        compaction_times_limit=rng.choice([1, 2, 3, 3, 4, 6] if not producer else [1, 2, 3]),
                        max_crash_times=rng.randint(0, 2 if not producer else 1),
                        consume_times_limit=rng.randint(0, 2), model_consumer=rng.random() < 0.3,
                        model_producer=producer, retain_null_key=rng.random() < 0.6, key_space=keys,
                        value_space=values, invariants=rng.sample(INVARIANTS, rng.randint(1, 4)),
                        check_deadlock=rng.random() < 0.8)


@pytest.mark.parametrize("seed", range(40))
def test_random_cfg_matches_oracle(seed):
    m = random_model(seed)
    if tlcgpu.check_model(m) is not None:
        pytest.skip(f"constants refused: {tlcgpu.check_model(m)}")
    want = run_oracle(m)
    for mode in ("auto", "tlc_order"):
        ck = tlcgpu.Checker(m, tlc_order=mode == "tlc_order", engine="auto" if mode == "auto" else "global",
                            outdegree=True)
        try:
            r = ck.run()
            assert r.status == want["result"], (seed, mode, r.status, want["result"])
            if want["result"] == "ok":
                assert (r.generated, r.distinct, r.depth, r.levels) == \
                       (want["generated"], want["distinct"], want["depth"], want["levels"]), (seed, mode)
                if mode == "tlc_order" or r.engine == "component":  # TLC's first-discoverer tree
                    assert ck.outdegree() == want["outdegree"], (seed, mode)
                continue
            assert r.depth == want["depth"], (seed, mode)
            if want["result"] in ("invariant", "invariant_error"):
                assert r.invariant == want["invariant"], (seed, mode)
            if mode == "tlc_order" or r.engine == "component":  # TLC's -workers 1 trace
                assert [tlcgpu.decode(m, s) for _, s in r.trace] == [t["state"] for t in want["trace"]], (seed, mode)
            if mode == "tlc_order":
                assert ck.tlc_stop_stats() == (want["generated"], want["distinct"], want["left_on_queue"]), seed
        finally:
            ck.close()
