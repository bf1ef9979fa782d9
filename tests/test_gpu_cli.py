"""GPU: the drop-in `tlc-hip` end to end on an MI355X, full stdout and exit
code, in built-in-module mode (no .tla on the box: the definitions' body
fingerprints and source extents of compaction.tla are compiled into the
binary, host/known_defs.inc).  The expected report is assembled from the
golden fixtures (oracle counts, TLC-syntax trace states) and from SURVEY 3.4's
action extents (compaction.tla:94-182).  [TLC-ext]: the message text follows
TLC's; it is not pinned by a TLC run."""
import os
import re
import subprocess

import pytest

from conftest import CLI, GOLDEN
from test_cli import numeric_cfg

pytestmark = pytest.mark.gpu

# "<Action line L1, col C1 to line L2, col C2 of module compaction>"
EXTENT = {
    "Producer": (84, 5, 87, 71),
    "CompactorPhaseOne": (94, 5, 100, 84),
    "CompactorPhaseTwoWrite": (122, 5, 132, 106),
    "CompactorPhaseTwoUpdateContext": (136, 5, 139, 77),
    "CompactorPhaseTwoUpdateHorizon": (142, 5, 145, 81),
    "CompactorPhaseTwoPersistCusror": (148, 5, 151, 116),
    "CompactorPhaseTwoDeleteLedger": (154, 5, 165, 90),
    "BrokerCrash": (170, 5, 182, 45),
    "Consumer": (186, 5, 186, 18),
    "Terminating": (207, 5, 214, 21),
}
DATE = re.compile(r"\d{4}-\d\d-\d\d \d\d:\d\d:\d\d")


def run(tmp_path, cfg_text, args=()):
    cfg = tmp_path / "m.cfg"
    cfg.write_text(cfg_text)
    p = subprocess.run([CLI, "-config", str(cfg)] + list(args), capture_output=True, text=True, timeout=300,
                       cwd=str(tmp_path))
    out = DATE.sub("<DATE>", p.stdout)
    out = re.sub(r"Finished in \d+s at", "Finished in <T> at", out)
    return p.returncode, out.splitlines()


def prob(p):  # Java-like "3.8E-11"
    import math
    e = math.floor(math.log10(p))
    m = p / 10 ** e
    if m >= 9.95:
        m, e = m / 10, e + 1
    return f"{m:.1f}E{e}"


def outdegree_line(hist):
    """TLC's BucketStatistics: rounded mean, minimum, maximum, the first bucket
    whose cumulative count reaches 95 %"""
    total = sum(hist)
    mean = round(sum(k * c for k, c in enumerate(hist)) / total)
    mn = next(k for k, c in enumerate(hist) if c)
    cum, p95 = 0, 0
    for k, c in enumerate(hist):
        cum += c
        if cum >= 0.95 * total:
            p95 = k
            break
    return (f"The average outdegree of the complete state graph is {mean} (minimum is {mn}, the maximum "
            f"{len(hist) - 1} and the 95th percentile is {p95}).")


def header(gpus=1):
    run_line = ("Running breadth-first search Model-Checking with 1 GPU (device 0) and seed 0." if gpus == 1 else
                f"Running breadth-first search Model-Checking with {gpus} GPU ranks (FPSet partitioned by owner, "
                f"rank r on device r mod 1) and seed 0.")
    return ["tlc-hip: TLC-compatible breadth-first model checking on MI355X (libtlcgpu ABI 4)", run_line,
            "Parsing file compaction.tla (built-in: the definitions of compaction.tla this build implements)",
            "Semantic processing of module compaction", "Starting... (<DATE>)", "Computing initial states..."]


@pytest.mark.parametrize("gpus", [1, 2])
def test_cli_shipped_numeric_cfg(tmp_path, gpus):
    """S: the summary, the collision estimate, the outdegree line, depth 20"""
    want = GOLDEN["S"]["result"]
    rc, lines = run(tmp_path, numeric_cfg(), ["-gpus", str(gpus)] if gpus > 1 else [])
    g, d = want["generated"], want["distinct"]
    expect = header(gpus) + [
        "Finished computing initial states: 729 distinct states generated at <DATE>.",
        "Model checking completed. No error has been found.",
        "  Estimates of the probability that TLC did not check all reachable states",
        "  because two distinct states had the same fingerprint:",
        f"  calculated (optimistic):  val = {prob(d * (g - d) / 2 ** 64)}",
        "  (tlc-hip keeps the packed states themselves: its FPSet is exact, actual collision probability 0)",
        f"{g} states generated, {d} distinct states found, 0 states left on queue.",
        "The depth of the complete state graph search is 20.",
    ]
    if gpus == 1:  # (TLC's first-discoverer parents: one context)
        expect.append(outdegree_line(want["outdegree"]))
    expect.append("Finished in <T> at (<DATE>)")
    assert rc == 0
    assert lines == expect


@pytest.mark.parametrize("case,code", [("V_leak", 12), ("V_dup", 12)])
def test_cli_counterexample(tmp_path, case, code):
    """a bug reproducer (compaction.cfg:27-31): TLC's -workers 1 trace with
    every state's action extent, TLC's counts where it stops, the exit code"""
    g = GOLDEN[case]
    want = g["result"]
    rc, lines = run(tmp_path, numeric_cfg(INVARIANTS=", ".join(g["constants"]["invariants"])))
    expect = header() + ["Finished computing initial states: 729 distinct states generated at <DATE>.",
                         f"Error: Invariant {want['invariant']} is violated.",
                         "Error: The behavior up to this point is:"]
    for i, t in enumerate(want["trace"]):
        if t["action"] == "Init":
            expect.append(f"State {i + 1}: <Initial predicate>")
        else:
            l0, c0, l1, c1 = EXTENT[t["action"]]
            expect.append(f"State {i + 1}: <{t['action']} line {l0}, col {c0} to line {l1}, col {c1} of module "
                          f"compaction>")
        expect += t["state"].split("\n") + [""]
    expect += [f"{want['generated']} states generated, {want['distinct']} distinct states found, "
               f"{want['left_on_queue']} states left on queue.",
               f"The depth of the complete state graph search is {want['depth']}.",
               "Finished in <T> at (<DATE>)"]
    assert rc == code
    assert lines == expect
    assert len(want["trace"]) == (12 if case == "V_leak" else 4)


def test_cli_shipped_string_keys_assume(tmp_path):
    """the shipped cfg binds KeySpace = {"key1", "key2"} (compaction.cfg:7):
    TLC stops on the ASSUME (compaction.tla:25-35) before any state"""
    rc, lines = run(tmp_path, numeric_cfg(KeySpace='{"key1", "key2"}'))
    assert rc == 75
    text = "\n".join(lines)
    assert "Evaluating assumption line 25, col 8 to line 35, col 35 of module compaction failed." in text
    assert 'Attempted to check if the value:\n"key1"\nis an element of Nat.' in text
    assert "Computing initial states..." not in text


def test_cli_termination_property(tmp_path):
    """PROPERTY Termination (compaction.tla:303-307) under Spec: the GPU
    liveness pass after the safety search; Spec has no fairness, so the
    counterexample is the first initial state in Init order followed by
    stuttering, exit code 13 ([TLC-ext] text)"""
    import tlcgpu
    from conftest import model_of
    want = GOLDEN["S"]["result"]
    rc, lines = run(tmp_path, numeric_cfg(PROPERTY="Termination"))
    assert rc == 13
    m = model_of(GOLDEN["S"]["constants"])
    first = tlcgpu.decode(m, tlcgpu.host_init_state(m, 0)).split("\n")
    i = lines.index(f"Checking temporal properties for the complete state space with {want['distinct']} total "
                    f"distinct states at (<DATE>)")
    assert re.fullmatch(r"Finished checking temporal properties in \d+s at <DATE>", lines[i + 1])
    assert lines[i + 2:i + 8] == ["Error: Temporal properties were violated.", "",
                                  "Error: The following behavior constitutes a counter-example:", "",
                                  "State 1: <Initial predicate>", first[0]]
    j = i + 7 + len(first)
    assert lines[i + 8:j] == first[1:] and lines[j:j + 2] == ["", "State 2: Stuttering"]
    assert f"{want['generated']} states generated, {want['distinct']} distinct states found, 0 states left on queue." in lines


@pytest.mark.parametrize("gpus", [1, 2])
def test_cli_injected_invariant(tmp_path, gpus):
    """BASELINE config 5: an invariant added to the module (here with -defs, as
    the box has no .tla) and named in INVARIANTS, violated at depth 12: TLC's
    -workers 1 trace, its counts where it stops, exit code 12 -- the Python
    oracle's fixture (tests/golden/user_inv.json, oracle/tla_eval.py).  With
    -gpus 2 the check runs on two ranks (the added invariant on both, VERDICT
    r4 item 2), and the report is the same TLC -workers 1 report."""
    import json
    from user_inv_cases import CASES
    g = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "user_inv.json")))
    want = g["U_LedgerCount"]["result"]
    defs = tmp_path / "added.tla"
    defs.write_text("\\* an invariant the user adds\nLedgerCount == " + CASES["LedgerCount"] + "\n")
    rc, lines = run(tmp_path, numeric_cfg(INVARIANTS="LedgerCount"),
                    ["-defs", str(defs)] + (["-gpus", str(gpus)] if gpus > 1 else []))
    expect = header(gpus) + ["Finished computing initial states: 729 distinct states generated at <DATE>.",
                         "Error: Invariant LedgerCount is violated.",
                         "Error: The behavior up to this point is:"]
    for i, t in enumerate(want["trace"]):
        if t["action"] == "Init":
            expect.append(f"State {i + 1}: <Initial predicate>")
        else:
            l0, c0, l1, c1 = EXTENT[t["action"]]
            expect.append(f"State {i + 1}: <{t['action']} line {l0}, col {c0} to line {l1}, col {c1} of module "
                          f"compaction>")
        expect += t["state"].split("\n") + [""]
    expect += [f"{want['generated']} states generated, {want['distinct']} distinct states found, "
               f"{want['left_on_queue']} states left on queue.",
               f"The depth of the complete state graph search is {want['depth']}.",
               "Finished in <T> at (<DATE>)"]
    assert rc == 12
    assert lines == expect
    assert len(want["trace"]) == 12
