"""CPU property test ("Property"): random walks from Init through
the product's packed semantics (model.h compiled for the host inside
libtlcgpu.so, the same code the gfx950 kernels run) in lockstep with the
independent pure-Python oracle (oracle/oracle_py.py, TEST INFRASTRUCTURE).

At every step of a walk the two must agree on: the successors in Next order
(action names and the TLC text of each state), evaluation errors, and the
first failing invariant (all four of compaction.tla:236-294, fixed order).
hypothesis draws the constants; wide (> 63-bit) layouts are included."""
import random

from hypothesis import HealthCheck, given, settings, strategies as st

import tlcgpu
from oracle_py import ACTIONS as PY_ACTIONS
from oracle_py import EvalError
from oracle_py import Model as PyModel

INVS = ("TypeSafe", "CompactedLedgerLeak", "CompactionHorizonCorrectness", "DuplicateNullKeyMessage")
PHASES = ("Compactor_In_PhaseOne", "Compactor_In_PhaseTwoWrite", "Compactor_In_PhaseTwoUpdateContext",
          "Compactor_In_PhaseTwoUpdateHorizon", "Compactor_In_PhaseTwoPersistCusror",
          "Compactor_In_PhaseTwoDeleteLedger")


def fmt_msg(m):
    return f"[id |-> {m[0]}, key |-> {m[1]}, value |-> {m[2]}]"


def fmt(s):
    """TLC's text of an oracle_py state: variables in declaration order
    (compaction.tla:57-70), record fields sorted, latestForKey as a tuple
    when its domain is 1..n (SURVEY App.C)."""
    msgs, led, cur, ph, p1r, hz, ctx, crash, cons = s
    out = ["/\\ messages = <<" + ", ".join(fmt_msg(m) for m in msgs) + ">>",
           "/\\ compactedLedgers = <<" + ", ".join(
               "Nil" if l is None else "<<" + ", ".join(fmt_msg(m) for m in l) + ">>" for l in led) + ">>",
           "/\\ cursor = " + ("Nil" if cur is None else
                              f"[compactedTopicContext |-> {cur[1]}, compactionHorizon |-> {cur[0]}]"),
           "/\\ compactorState = " + PHASES[ph]]
    if p1r is None:
        out.append("/\\ phaseOneResult = Nil")
    else:
        rp, latest = p1r
        keys = [k for k, _ in latest]
        if keys == list(range(1, len(keys) + 1)):
            lf = "<<" + ", ".join(str(v) for _, v in latest) + ">>"
        else:
            lf = "(" + " @@ ".join(f"{k} :> {v}" for k, v in latest) + ")"
        out.append(f"/\\ phaseOneResult = [latestForKey |-> {lf}, readPosition |-> {rp}]")
    out += [f"/\\ compactionHorizon = {hz}", f"/\\ compactedTopicContext = {ctx}", f"/\\ crashTimes = {crash}",
            f"/\\ consumeTimes = {cons}"]
    return "\n".join(out)


def py_first_failing(py, s):
    """-1, or (index << 1) | is_error, like tlcg_host_check_invariants."""
    for q, name in enumerate(INVS):
        try:
            if not py.inv(name, s):
                return q << 1
        except EvalError:
            return (q << 1) | 1
    return -1


CONSTS = st.fixed_dictionaries(dict(
    N=st.integers(0, 4), C=st.integers(1, 7), K=st.integers(0, 2),
    keys=st.lists(st.integers(1, 9), max_size=3, unique=True),
    values=st.lists(st.integers(1, 9), max_size=2, unique=True),
    retain=st.booleans(), producer=st.booleans(), consumer=st.booleans(), ctl=st.integers(0, 2)))


@settings(max_examples=150, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(c=CONSTS, seed=st.integers(0, 2 ** 32 - 1))
def test_random_walk_matches_oracle(c, seed):
    m = tlcgpu.Model(msg_sent_limit=c["N"], compaction_times_limit=c["C"], max_crash_times=c["K"],
                     consume_times_limit=c["ctl"], model_consumer=c["consumer"], model_producer=c["producer"],
                     retain_null_key=c["retain"], key_space=c["keys"], value_space=c["values"], invariants=INVS)
    assert tlcgpu.check_model(m) is None  # every drawn layout packs into <= 126 bits
    py = PyModel(N=c["N"], C=c["C"], K=c["K"], keys=c["keys"], values=c["values"], retain=c["retain"],
                 producer=c["producer"], consumer=c["consumer"], ctl=c["ctl"], invariants=INVS)
    rnd = random.Random(seed)
    inits = list(py.inits())
    assert len(inits) == tlcgpu.init_count(m)
    i = rnd.randrange(len(inits))
    s_py, s = inits[i], tlcgpu.host_init_state(m, i)
    for _ in range(80):
        assert tlcgpu.decode(m, s) == fmt(s_py)
        assert tlcgpu.host_check_invariants(m, s) == py_first_failing(py, s_py)
        try:
            succ_py = list(py.successors(s_py))
        except EvalError:
            succ_py = None
        try:
            succ = tlcgpu.host_successors(m, s)
        except RuntimeError:
            succ = None
        assert (succ is None) == (succ_py is None)
        if not succ:
            break
        assert [a for a, _ in succ] == [PY_ACTIONS[a] for a, _ in succ_py]
        assert [tlcgpu.decode(m, t) for _, t in succ] == [fmt(t) for _, t in succ_py]
        j = rnd.randrange(len(succ))
        s, s_py = succ[j][1], succ_py[j][1]
