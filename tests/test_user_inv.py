"""User invariants (BASELINE config 5: an invariant injected into
compaction.tla), CPU side: the product's compiler + interpreter
(user_inv.{h,cpp}, run through tlcg_host_check_invariants_batch) against the
oracle's independent parser/evaluator (oracle/tla_eval.py) on every reachable
state, the spec's own invariants compiled from the reference's TLA+ text
against the hand-written evaluators, and the refusals."""
import os

import pytest

from user_inv_cases import (CASES, HELPERS, REF_TLA, T, model_with, oracle_model, paired_states, ref_definition,
                            semantic_mutants)


def oracle_code(om, names, s):
    """the oracle's first failing invariant, as check_invariants encodes it"""
    import oracle_py
    for q, n in enumerate(names):
        try:
            if not om.inv(n, s):
                return q << 1
        except oracle_py.EvalError:
            return (q << 1) | 1
    return -1


# (cfg, stride): every reachable state of the shipped constants; every 3rd of the others
CONFIGS = {
    "S": (dict(), 1),
    "S-noretain": (dict(retain_null_key=False), 3),
    "S-C2K2": (dict(compaction_times_limit=2, max_crash_times=2), 3),
    "P-producer": (dict(model_producer=True, key_space=(1,), value_space=(1,)), 3),
    "S-keys59": (dict(key_space=(5, 9), value_space=(7,)), 3),
}


@pytest.mark.parametrize("cfg", sorted(CONFIGS))
def test_user_invariants_match_oracle_on_every_reachable_state(cfg):
    kw, stride = CONFIGS[cfg]
    names = sorted(CASES)
    base = T.Model(**kw)
    pairs = paired_states(base)[::stride]
    words = [w for w, _ in pairs]
    om = oracle_model(model_with(names, **kw))
    # the oracle's verdict of each invariant on each state
    want = {n: [] for n in names}
    for _, o in pairs:
        for n in names:
            want[n].append(oracle_code(om, [n], o))
    disagreements = []
    for n in names:  # one invariant at a time
        got = T.host_check_invariants_batch(model_with([n], **kw), words)
        disagreements += [(n, T.decode(base, w), g, x) for (w, _), g, x in zip(pairs, got, want[n]) if g != x]
    assert not disagreements, disagreements[:5]
    # several in one cfg list (at most 8): the first failing one in cfg order
    for chunk in (names[:8], names[8:], names[::-1][:8]):
        got = T.host_check_invariants_batch(model_with(chunk, **kw), words)
        first = []
        for i in range(len(pairs)):
            codes = [want[n][i] for n in chunk]
            q = next((q for q, c in enumerate(codes) if c >= 0), None)
            first.append(-1 if q is None else (q << 1) | (codes[q] & 1))
        assert got == first


def test_user_invariants_exercise_every_outcome():
    """the cases reach TRUE, FALSE and evaluation errors on the shipped constants"""
    pairs = paired_states(T.Model())
    words = [w for w, _ in pairs]
    outcomes = {}
    for n in CASES:
        got = set(T.host_check_invariants_batch(model_with([n]), words))
        outcomes[n] = got
    assert any(0 in g for g in outcomes.values())   # violated somewhere
    assert any(1 in g for g in outcomes.values())   # an evaluation error somewhere
    assert all(-1 in g for g in outcomes.values())  # each holds somewhere
    assert outcomes["LedgerCount"] == {-1, 0}
    assert outcomes["ContextLedgerError"] == {1} or 1 in outcomes["ContextLedgerError"]


@pytest.mark.skipif(not os.path.exists(REF_TLA), reason="the reference spec is read at test time")
@pytest.mark.parametrize("cfg", ["S", "S-noretain", "P-producer", "S-C2K2"])
def test_spec_invariants_compiled_from_the_reference_text(cfg):
    """TypeSafe, CompactedLedgerLeak, CompactionHorizonCorrectness and
    DuplicateNullKeyMessage (compaction.tla:236-294) read from the reference
    .tla and compiled as user invariants give the hand-written evaluators'
    verdict (model.h, pinned by the oracles) on every reachable state"""
    kw = CONFIGS[cfg][0]
    defs = {}
    for name in ("NullKey", "NullValue", "KeySet", "ValueSet", "CompactorState", "Max", "GetKeys",
                 "MaxCompactedLedgerId"):
        params, body = ref_definition(name)
        defs[name + params] = body
    builtin = ("TypeSafe", "CompactedLedgerLeak", "CompactionHorizonCorrectness", "DuplicateNullKeyMessage")
    for name in builtin:
        _, body = ref_definition(name)
        defs["User" + name] = body
    pairs = paired_states(T.Model(**kw))
    words = [w for w, _ in pairs]
    for name in builtin:
        want = T.host_check_invariants_batch(T.Model(invariants=(name,), **kw), words)
        got = T.host_check_invariants_batch(T.Model(invariants=("User" + name,), user_defs=defs, **kw), words)
        assert got == want, name
    # all four in one cfg list, user versions
    users = tuple("User" + n for n in builtin)
    want = T.host_check_invariants_batch(T.Model(invariants=builtin, **kw), words)
    got = T.host_check_invariants_batch(T.Model(invariants=users, user_defs=defs, **kw), words)
    assert got == want


REFUSED = {
    "Primed": ("compactionHorizon' = 0", "primed"),
    "Except": ("[compactedLedgers EXCEPT ![1] = Nil] = compactedLedgers", "EXCEPT"),
    "Subset": ("SUBSET KeySpace # {}", "SUBSET"),
    "Unknown": ("frobnicate > 0", "unknown identifier frobnicate"),
    "NotBool": ("compactionHorizon + 1", "not a boolean"),
    "IntVsBool": ("compactionHorizon = TRUE", "cannot compare"),
    "Strings": ("\"key1\" \\in KeySpace", "strings"),
    "Recursive": ("Recursive", "nest too deeply"),
}


@pytest.mark.parametrize("name", sorted(REFUSED))
def test_unsupported_invariants_are_refused_with_a_reason(name):
    body, why = REFUSED[name]
    m = T.Model(invariants=(name,), user_defs={name: body})
    err = T.check_model(m)
    assert err is not None and why in err and name in err, err


def test_bulleted_lists_are_read_by_column():
    # the second /\ at a smaller column ends the inner list (TLA+'s offside rule)
    body = ("/\\ compactionHorizon <= 3\n"
            "/\\ \\/ compactedTopicContext = 0\n"
            "   \\/ compactedTopicContext >= 1\n"
            "/\\ crashTimes <= 1")
    m = T.Model(invariants=("Bullets",), user_defs={"Bullets": body})
    assert T.check_model(m) is None
    s = T.host_init_state(m, 0)
    assert T.host_check_invariants(m, s) == -1
    bad = T.Model(invariants=("Bullets",), user_defs={"Bullets": body.replace("<= 1", "> 1")})
    assert T.host_check_invariants(bad, s) == 0


def test_user_definition_shadows_a_spec_invariant_name():
    m = T.Model(invariants=("TypeSafe",), user_defs={"TypeSafe": "FALSE"})
    assert T.host_check_invariants(m, T.host_init_state(m, 0)) == 0


def _golden_user():
    import json
    return json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "user_inv.json")))


def _golden_model(case):
    g = _golden_user()[case]
    return T.Model(invariants=tuple(g["invariants"]), user_defs=g["user_defs"], **g["constants"])


@pytest.mark.parametrize("case", ["U_all_hold", "U_LedgerCount", "U_ArithCase", "U_C5K2_MaxLedgerBound",
                                  "U_producer_LedgerCount", "U_KeysKnown"])
def test_user_invariants_compile_into_the_specialized_kernels(case):
    """the program lowered to device code (user_inv.cpp user_device_source)
    compiles with the component and tree kernels for gfx950 without a device
    (a failure would leave the model to the global engine at run time)"""
    import ctypes as C
    m = _golden_model(case).to_c()
    err = C.create_string_buffer(8192)
    n = T.load_library().tlcg_jit_selftest(C.byref(m), b"gfx950", err, 8192)
    assert n > 0, err.value.decode()[:3000]


def test_user_invariant_views_agree_on_every_reachable_state():
    """the on-chip engines evaluate a user invariant on their own encoding
    (component_code.h UVCode: a component code plus the component's
    constants); on every reachable state of 200 components of each
    non-producer golden cfg, every field it reads and every invariant's
    outcome equal the packed word's (model.h UVWord), narrow and wide"""
    for case, g in sorted(_golden_user().items()):
        m = _golden_model(case)
        if m.model_producer:
            continue
        assert T.host_component_selfcheck(m, 0, 200) > 0, case
    wide = T.Model(invariants=("LedgerCount",), user_defs={"LedgerCount": CASES["LedgerCount"]},
                   compaction_times_limit=12, key_space=range(1, 4), value_space=range(1, 4))
    assert T.state_words(wide) == 2 and T.host_component_selfcheck(wide, 0, 12) > 0


def test_integer_overflow_is_an_evaluation_error():
    """TLC's integers are 32-bit: an arithmetic result outside -2^31..2^31-1
    is an evaluation error ([TLC-ext] the overflow check of TLC's Naturals /
    Integers), never a wrapped or 64-bit value; parity unpinned against TLC"""
    s = T.host_init_state(T.Model(), 0)
    big = T.Model(invariants=("Big",), user_defs={"Big": "2147483647 + crashTimes + 1 > 0"})
    assert T.host_check_invariants(big, s) == 1  # (index 0 << 1) | error
    ok = T.Model(invariants=("Fits",), user_defs={"Fits": "2147483646 + crashTimes + 1 > 0"})
    assert T.host_check_invariants(ok, s) == -1
    mul = T.Model(invariants=("Mul",), user_defs={"Mul": "65536 * 65536 + crashTimes >= 0"})
    assert T.host_check_invariants(mul, s) == 1


# ---- differential mutation test: semantic mutants of every fixture body
# (user_inv_cases.semantic_mutants) compiled by the product and by the
# oracle's independent evaluator, compared on every reachable state of a
# small model wherever both accept the mutant
def test_semantic_mutants_match_the_oracle():
    import random
    rng = random.Random(20261017)
    kw = dict(msg_sent_limit=2, compaction_times_limit=2)
    pairs = paired_states(T.Model(**kw))
    words = [w for w, _ in pairs]
    compared = disagreements = 0
    bad = []
    for name in sorted(CASES):
        for body in semantic_mutants(CASES[name], rng, 24):
            defs = dict(HELPERS)
            defs[name] = body
            m = T.Model(invariants=(name,), user_defs=defs, **kw)
            try:
                got = T.host_check_invariants_batch(m, words)
            except ValueError:
                continue  # refused by the product (outside its subset, or a type error)
            om = oracle_model(m)
            try:
                want = [oracle_code(om, [name], o) for _, o in pairs]
            except Exception:  # noqa: BLE001  (outside the oracle evaluator's subset)
                continue
            compared += 1
            diff = [(T.decode(T.Model(**kw), w), g, x) for (w, _), g, x in zip(pairs, got, want) if g != x]
            if diff:
                disagreements += 1
                bad.append((name, body, diff[:2]))
    assert not bad, (compared, bad[:3])
    assert compared >= 100, compared
