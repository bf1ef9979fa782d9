"""CPU: the oracle against the reference's published numbers, SURVEY's hand
derivations, the committed golden fixtures and the second (Python) oracle."""
import pytest

from conftest import FULL_CASES, GOLDEN, model_of, run_oracle
from oracle_py import Model as PyModel


def test_published_45198():
    # compaction.tla:23 -- "if disable modelling of consumer and producer ... 45198"
    r = run_oracle(model_of(GOLDEN["S"]["constants"]))
    assert r["result"] == "ok" and r["distinct"] == 45198


def test_published_253361():
    # compaction.tla:23 -- "... decrease from 253361": producer modelled; the
    # number is reproduced with RetainNullKey = FALSE (consumer is a pure stutter)
    for case in ("P_published", "P_published_consumer"):
        r = run_oracle(model_of(GOLDEN[case]["constants"]))
        assert r["result"] == "ok" and r["distinct"] == 253361


def test_survey_app_a2_shipped_numeric():
    # SURVEY.md App.A.2: 729 x 62 distinct, 729 x 83 generated, depth 20, per-level law
    r = run_oracle(model_of(GOLDEN["S"]["constants"]))
    per_m = [1, 2, 2, 3, 3, 3, 4, 3, 3, 4, 4, 3, 4, 4, 4, 5, 5, 1, 2, 2]
    assert r["generated"] == 60507 and r["depth"] == 20
    assert r["levels"] == [729 * x for x in per_m]


def test_survey_app_a3_scaling_law():
    for C in range(1, 7):
        assert GOLDEN[f"R_C{C}_K0"]["result"]["distinct"] == 6 * C + 2
        assert GOLDEN[f"R_C{C}_K0"]["result"]["depth"] == 6 * C + 2
        want = 18 if C == 1 else 3 * C * C + 10 * C + 5
        assert GOLDEN[f"R_C{C}_K1"]["result"]["distinct"] == want


def test_survey_app_a4_counterexamples():
    leak = GOLDEN["V_leak"]["result"]
    assert leak["result"] == "invariant" and leak["invariant"] == "CompactedLedgerLeak"
    assert [t["action"] for t in leak["trace"]] == [
        "Init", "CompactorPhaseOne", "CompactorPhaseTwoWrite", "CompactorPhaseTwoUpdateContext",
        "CompactorPhaseTwoUpdateHorizon", "CompactorPhaseTwoPersistCusror", "CompactorPhaseTwoDeleteLedger",
        "CompactorPhaseOne", "CompactorPhaseTwoWrite", "BrokerCrash", "CompactorPhaseOne",
        "CompactorPhaseTwoWrite"]
    dup = GOLDEN["V_dup"]["result"]
    assert dup["invariant"] == "DuplicateNullKeyMessage" and len(dup["trace"]) == 4
    # the first initial state in TLC order is the all-null message sequence M0
    assert "key |-> 0, value |-> 0], [id |-> 2, key |-> 0" in leak["trace"][0]["state"]


@pytest.mark.parametrize("case", FULL_CASES)
def test_golden_reproducible(case):
    g = GOLDEN[case]
    r = run_oracle(model_of(g["constants"]))
    r.pop("seconds", None)
    want = dict(g["result"])
    want.pop("seconds", None)
    assert r == want


def test_per_m_isomorphism():
    # every message sequence M has the same compactor graph (SURVEY App.A.1):
    # 100 consecutive Ms of G9 give exactly 100 x the first M's counts
    one, many = GOLDEN["G9_first_M"]["result"], GOLDEN["G9_some_M"]["result"]
    assert many["distinct"] == 100 * one["distinct"] and many["generated"] == 100 * one["generated"]
    assert many["levels"] == [100 * x for x in one["levels"]]


@pytest.mark.parametrize("case", ["S", "X_keys3_vals57", "X_producer_sparse", "V_leak", "V_dup", "D_N0_K1",
                                  "R_C4_K2", "S_consumer"])
def test_python_oracle_agrees(case):
    c = GOLDEN[case]["constants"]
    p = PyModel(N=c["N"], C=c["C"], K=c["K"], keys=c["keys"], values=c["values"], retain=c["retain"],
                producer=c["producer"], consumer=c["consumer"], ctl=c["ctl"], invariants=c["invariants"],
                deadlock=c["deadlock"]).check()
    g = GOLDEN[case]["result"]
    assert p["result"] == g["result"]
    if g["result"] == "ok":
        assert (p["generated"], p["distinct"], p["depth"], p["levels"]) == (g["generated"], g["distinct"],
                                                                            g["depth"], g["levels"])
    else:
        assert [a for a, _ in p["trace"]] == [t["action"] for t in g["trace"]]
