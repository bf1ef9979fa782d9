"""Regenerate tests/golden/golden.json from the CPU oracle (oracle/build/tlc_oracle).

Every case is also run through the independent pure-Python oracle
(oracle/oracle_py.py) when small enough, and the two must agree before a
fixture is written.  The two numbers the reference publishes
(/root/reference/compaction.tla:23: 253361 and 45198) are asserted here.

    python tests/golden/make_golden.py
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
from oracle_py import Model as PyModel  # noqa: E402

ORACLE = os.path.join(ROOT, "oracle", "build", "tlc_oracle")
INV2 = ["TypeSafe", "CompactionHorizonCorrectness"]

# name -> constants (defaults: the shipped compaction.cfg with numeric keys)
BASE = dict(N=3, C=3, K=1, keys=[1, 2], values=[1, 2], retain=True, producer=False, consumer=False, ctl=2,
            invariants=INV2, deadlock=True)
CASES = {
    # the shipped cfg with KeySpace = {1, 2}: published 45198 (compaction.tla:23)
    "S": dict(),
    "S_noretain": dict(retain=False),
    # producer (+consumer) modelled: published 253361 (compaction.tla:23) at RetainNullKey = FALSE
    "P_published": dict(producer=True, retain=False),
    "P_published_consumer": dict(producer=True, consumer=True, retain=False),
    "P_retain_consumer": dict(producer=True, consumer=True, retain=True),
    "S_consumer": dict(consumer=True),
    "S_consumer_ctl0": dict(consumer=True, ctl=0),
    # the spec's bug reproducers (compaction.cfg:27-31) -> counterexamples
    "V_leak": dict(invariants=["TypeSafe", "CompactedLedgerLeak", "CompactionHorizonCorrectness"]),
    "V_dup": dict(invariants=["TypeSafe", "CompactionHorizonCorrectness", "DuplicateNullKeyMessage"]),
    "V_leak_producer": dict(producer=True, retain=False, invariants=["CompactedLedgerLeak"]),
    "V_dup_producer": dict(producer=True, invariants=["DuplicateNullKeyMessage"]),
    # deadlock: MessageSentLimit = 0 leaves only BrokerCrash
    "D_N0_K1": dict(N=0, K=1),
    "D_N0_K0": dict(N=0, K=0),
    "D_N0_K1_nodeadlock": dict(N=0, K=1, deadlock=False),
    # other shapes: non-contiguous spaces, more crashes, more compactions
    "X_keys3_vals57": dict(N=2, C=2, K=2, keys=[1, 2, 3], values=[5, 7]),
    "X_producer_sparse": dict(N=2, C=2, K=1, keys=[3, 9], values=[4], producer=True),
    "X_C5_K2": dict(N=2, C=5, K=2, keys=[1], values=[1]),
    "X_empty_spaces": dict(N=3, C=3, K=1, keys=[], values=[]),
}
# wide layouts (> 63 bits: two-word states, SURVEY 8(d) G9-deep family)
CASES.update({
    "W_C12_k1": dict(C=12, keys=[1], values=[1]),
    "W_C12": dict(C=12),
    "W_C12_noretain": dict(C=12, retain=False),
    "W_C12_leak": dict(C=12, keys=[1], values=[1], invariants=["TypeSafe", "CompactedLedgerLeak"]),
    "W_C12_dup": dict(C=12, keys=[1], values=[1], invariants=["DuplicateNullKeyMessage"]),
    "W_P_C12": dict(C=12, keys=[1], values=[1], producer=True, retain=False),
    "W_N4_C6": dict(N=4, C=6, keys=[1, 2, 3], values=[1]),
    "W_N4_C6_K2_consumer": dict(N=4, C=6, K=2, keys=[1, 2, 3], values=[1], consumer=True, ctl=0),
})
# one M of G9-deep (KeySpace = ValueSpace = {1..10}, CompactionTimesLimit = 12)
CASES["G9deep_first_M"] = dict(C=12, keys=list(range(1, 11)), values=list(range(1, 11)), init_range=[0, 1])
CASES["G9deep_some_M"] = dict(C=12, keys=list(range(1, 11)), values=list(range(1, 11)), init_range=[777000, 777050])
# R(C, K): one initial state (KeySpace = ValueSpace = {}), N = 1
for C in range(1, 7):
    for K in range(0, 4):
        CASES[f"R_C{C}_K{K}"] = dict(N=1, C=C, K=K, keys=[], values=[])
# one M of the scaled configs (per-M counts; every M has the same graph, SURVEY App.A.1)
CASES["M8_first_M"] = dict(keys=list(range(1, 11)), values=list(range(1, 11)), init_range=[0, 1])
CASES["G9_first_M"] = dict(keys=list(range(1, 16)), values=list(range(1, 16)), init_range=[0, 1])
CASES["G9_some_M"] = dict(keys=list(range(1, 16)), values=list(range(1, 16)), init_range=[123456, 123556])


def oracle_args(c):
    a = ["-N", str(c["N"]), "-C", str(c["C"]), "-K", str(c["K"]), "-ctl", str(c["ctl"]),
         "-keys", ",".join(map(str, c["keys"])), "-values", ",".join(map(str, c["values"])),
         "-retain", str(int(c["retain"])), "-producer", str(int(c["producer"])),
         "-consumer", str(int(c["consumer"])), "-inv", ",".join(c["invariants"]), "-levels"]
    if not c["deadlock"]:
        a.append("-nodeadlock")
    if "init_range" in c:
        a += ["-init-lo", str(c["init_range"][0]), "-init-hi", str(c["init_range"][1])]
    return a


def run_oracle(c):
    out = subprocess.run([ORACLE] + oracle_args(c), check=True, capture_output=True, text=True).stdout
    return json.loads(out)


def py_check(c):
    m = PyModel(N=c["N"], C=c["C"], K=c["K"], keys=c["keys"], values=c["values"], retain=c["retain"],
                producer=c["producer"], consumer=c["consumer"], ctl=c["ctl"], invariants=c["invariants"],
                deadlock=c["deadlock"])
    return m.check()


def main():
    if not os.path.exists(ORACLE):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True)
    golden = {}
    for name, over in CASES.items():
        c = dict(BASE)
        c.update(over)
        r = run_oracle(c)
        if "init_range" not in c and r["distinct" if r["result"] == "ok" else "generated"] < 400000:
            p = py_check(c)
            assert p["result"] == r["result"], (name, p["result"], r["result"])
            if r["result"] == "ok":
                assert (p["generated"], p["distinct"], p["depth"], p["levels"], p["outdegree"]) == \
                       (r["generated"], r["distinct"], r["depth"], r["levels"], r["outdegree"]), name
            else:
                assert [a for a, _ in p["trace"]] == [t["action"] for t in r["trace"]], name
                # TLC's counters where the one-worker run stops
                assert (p["generated"], p["distinct"], p["left_on_queue"]) == \
                       (r["generated"], r["distinct"], r["left_on_queue"]), name
                # a level-synchronous checker's counts: the level that found the error finished
                assert (p["eol_generated"], p["eol_distinct"]) == (r["eol_generated"], r["eol_distinct"]), name
        golden[name] = dict(constants=c, result=r)
        if "init_range" not in c and r["result"] == "ok":
            # PROPERTY Termination (compaction.tla:303-307) under Spec and under
            # Spec /\ WF_vars(Next): the C oracle's Tarjan SCC restatement,
            # cross-checked against the Python oracle's DFS on small graphs
            live = {}
            for fair in ("none", "wf"):
                out = subprocess.run([ORACLE] + oracle_args(c) + ["-liveness", fair], check=True,
                                     capture_output=True, text=True).stdout
                lv = json.loads(out)
                lv.pop("stuck_trace", None)
                if lv["states_notp"] < 400000:
                    pl = PyModel(N=c["N"], C=c["C"], K=c["K"], keys=c["keys"], values=c["values"],
                                 retain=c["retain"], producer=c["producer"], consumer=c["consumer"],
                                 ctl=c["ctl"]).liveness(fair == "wf")
                    assert (pl["holds"], pl["states_notp"], pl["init_notp"], pl["edges_notp"], pl["stuck"],
                            pl["stuck_min_depth"], pl["cyclic"]) == \
                           (lv["holds"], lv["states_notp"], lv["init_notp"], lv["edges_notp"], lv["stuck"],
                            lv["stuck_min_depth"], lv["cyclic_sccs"] > 0), (name, fair, pl, lv)
                live[fair] = lv
            golden[name]["liveness"] = live
        print(f"{name:24s} {r['result']:10s} gen={r['generated']} distinct={r.get('distinct')} depth={r.get('depth')}")
    assert golden["S"]["result"]["distinct"] == 45198            # compaction.tla:23
    assert golden["P_published"]["result"]["distinct"] == 253361  # compaction.tla:23
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden.json"), "w") as f:
        json.dump(golden, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
