"""Regenerate tests/golden/user_inv.json: whole checks with user invariants
(BASELINE config 5: invariants injected into compaction.tla) by the Python
oracle, whose TLA+ evaluator is oracle/tla_eval.py.  The C oracle does not
evaluate user invariants, so these fixtures rest on the Python oracle alone;
its state rendering is checked against the C oracle's on a shared trace here,
and its evaluator against the product's on every reachable state in
tests/test_user_inv.py.

    python tests/golden/make_golden_user.py
"""
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.dirname(HERE))
import oracle_py  # noqa: E402
from user_inv_cases import CASES, HELPERS  # noqa: E402

ORACLE = os.path.join(ROOT, "oracle", "build", "tlc_oracle")

# name -> (constants as tlcgpu.Model keyword arguments, INVARIANTS)
RUNS = {f"U_{n}": (dict(), (n,)) for n in CASES}
RUNS.update({
    "U_mixed_builtin_first": (dict(), ("TypeSafe", "LedgerCount", "CompactionHorizonCorrectness")),
    "U_mixed_user_first": (dict(), ("ContextBound", "CompactedLedgerLeak")),
    "U_all_hold": (dict(), ("TypeSafe", "PhaseKnown", "LatestIsLast", "LedgerSorted", "KeysKnown", "MessageRec",
                            "HeadFirst", "CompactionHorizonCorrectness")),
    "U_producer_LedgerCount": (dict(model_producer=True, retain_null_key=False, key_space=(1,), value_space=(1, 2)),
                               ("TypeSafe", "LedgerCount")),
    "U_noretain_LatestIsLast": (dict(retain_null_key=False), ("LatestIsLast", "LedgerSorted")),
    "U_C5_ContextBound": (dict(compaction_times_limit=5, key_space=(1,), value_space=(1,)), ("ContextBound",)),
    "U_C5K2_MaxLedgerBound": (dict(compaction_times_limit=5, max_crash_times=2, key_space=(1,), value_space=(1,)),
                              ("MaxLedgerBound",)),
})


def oracle_model(kw, invariants):
    names = set(invariants)
    defs = dict(HELPERS)
    defs.update({n: CASES[n] for n in CASES if n in names})
    return oracle_py.Model(N=kw.get("msg_sent_limit", 3), C=kw.get("compaction_times_limit", 3),
                           K=kw.get("max_crash_times", 1), keys=list(kw.get("key_space", (1, 2))),
                           values=list(kw.get("value_space", (1, 2))), retain=kw.get("retain_null_key", True),
                           producer=kw.get("model_producer", False), consumer=False, ctl=2,
                           invariants=invariants, deadlock=True, user_defs=defs), defs


def main():
    # the Python oracle's rendering = the C oracle's, on a shared counterexample
    if not os.path.exists(ORACLE):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True)
    inv = ["TypeSafe", "CompactedLedgerLeak", "CompactionHorizonCorrectness"]
    c = json.loads(subprocess.run([ORACLE, "-inv", ",".join(inv)], check=True, capture_output=True,
                                  text=True).stdout)
    p = oracle_py.Model(invariants=inv).check()
    assert [oracle_py.Model.render(s) for _, s in p["trace"]] == [t["state"] for t in c["trace"]]

    golden = {}
    for name, (kw, invs) in RUNS.items():
        om, defs = oracle_model(kw, invs)
        r = om.check()
        if "trace" in r:
            r["trace"] = [dict(action=a, state=oracle_py.Model.render(s)) for a, s in r["trace"]]
            r["depth"] = len(r["trace"])
        golden[name] = dict(constants=kw, invariants=list(invs), user_defs=defs, result=r)
        print(f"{name:28s} {r['result']:16s} {r.get('invariant', '')}: gen={r['generated']} "
              f"distinct={r['distinct']} depth={r.get('depth')}")
    with open(os.path.join(HERE, "user_inv.json"), "w") as f:
        json.dump(golden, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
