"""ctypes binding of libtlcgpu.so (include/tlcgpu.h) -- the MI355X checker.

This is the Python face of the C ABI, used by bench.py, __graft_entry__ and the
tests.  It mirrors TLC's vocabulary: a `Model` is the constants a TLC cfg binds
(/root/reference/compaction.cfg:2-11) plus its INVARIANTS list (:25-31); a
`Checker` runs the breadth-first safety check and reports TLC's numbers.

There is no CPU fallback: if the HIP library is missing or no GPU is visible,
constructing a Checker raises.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("TLCG_LIB") or os.path.normpath(os.path.join(HERE, "..", "lib", "libtlcgpu.so"))

MAX_SET = 63
MAX_INV = 8

INVARIANTS = ("TypeSafe", "CompactedLedgerLeak", "CompactionHorizonCorrectness", "DuplicateNullKeyMessage")
INV_USER = 16  # TLCG_INV_USER: invariants[q] = INV_USER + j names the j-th user definition
ACTIONS = ("Producer", "CompactorPhaseOne", "CompactorPhaseTwoWrite", "CompactorPhaseTwoUpdateContext",
           "CompactorPhaseTwoUpdateHorizon", "CompactorPhaseTwoPersistCusror", "CompactorPhaseTwoDeleteLedger",
           "BrokerCrash", "Consumer", "Terminating")
STATUS = {0: "running", 1: "ok", 2: "invariant", 3: "deadlock", 4: "action_error", 5: "invariant_error"}
ENGINES = {"auto": 0, "global": 1, "component": 2, "tree": 3}
ENGINE_NAMES = {1: "global", 2: "component", 3: "tree"}


class tlcg_model(C.Structure):
    _fields_ = [("msg_sent_limit", C.c_int32), ("compaction_times_limit", C.c_int32),
                ("consume_times_limit", C.c_int32), ("max_crash_times", C.c_int32),
                ("model_consumer", C.c_uint8), ("model_producer", C.c_uint8),
                ("retain_null_key", C.c_uint8), ("check_deadlock", C.c_uint8),
                ("n_keys", C.c_int32), ("n_values", C.c_int32),
                ("keys", C.c_int64 * MAX_SET), ("values", C.c_int64 * MAX_SET),
                ("n_invariants", C.c_int32), ("invariants", C.c_int32 * MAX_INV),
                ("user_defs", C.c_char_p)]


class tlcg_opts(C.Structure):
    _fields_ = [("device", C.c_int32), ("log2_fpset_slots", C.c_int32), ("state_capacity", C.c_uint64),
                ("tlc_order", C.c_int32), ("rank", C.c_int32), ("world", C.c_int32), ("partition", C.c_int32),
                ("engine", C.c_int32), ("spill", C.c_int32), ("device_store_cap", C.c_uint64),
                ("fpset_spill", C.c_int32), ("log2_fpset_max", C.c_int32), ("outdegree", C.c_int32),
                ("reserved", C.c_int32 * 1)]


class tlcg_stats(C.Structure):
    _fields_ = [("generated", C.c_uint64), ("distinct", C.c_uint64), ("frontier", C.c_uint64),
                ("depth", C.c_int32), ("status", C.c_int32), ("invariant", C.c_int32), ("action", C.c_int32),
                ("event_gidx", C.c_uint64), ("fp_collision_optimistic", C.c_double), ("kernel_ms", C.c_double),
                ("expand_ms", C.c_double), ("levels_redone", C.c_uint64), ("engine", C.c_uint64),
                ("jit_used", C.c_uint64), ("host_states", C.c_uint64), ("fpset_host_states", C.c_uint64),
                ("transport", C.c_uint64), ("tlc_exact", C.c_uint64)]


class tlcg_liveness(C.Structure):
    _fields_ = [("holds", C.c_int32), ("kind", C.c_int32), ("fairness", C.c_int32), ("depth", C.c_int32),
                ("states_notp", C.c_uint64), ("init_notp", C.c_uint64), ("edges_notp", C.c_uint64),
                ("stuck", C.c_uint64), ("on_cycles", C.c_uint64), ("peel_rounds", C.c_uint64),
                ("trace_len", C.c_int32), ("loop_to", C.c_int32), ("back_action", C.c_int32),
                ("reserved", C.c_int32), ("kernel_ms", C.c_double), ("wall_ms", C.c_double)]


FAIRNESS = {"none": 0, "wf": 1}
LIVE_KINDS = {0: "holds", 1: "stuttering", 2: "cycle"}

_lib = None


def load_library(path: str = LIB_PATH):
    """Load libtlcgpu.so and declare every exported signature."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise RuntimeError(f"libtlcgpu.so not built at {path}: run __graft_entry__.build()")
    lib = C.CDLL(path)
    P, U64, I32 = C.c_void_p, C.c_uint64, C.c_int32
    M, O, S = C.POINTER(tlcg_model), C.POINTER(tlcg_opts), C.POINTER(tlcg_stats)
    sig = {
        "tlcg_abi_version": (C.c_int, []),
        "tlcg_check_model": (C.c_int, [M, C.c_char_p, I32]),
        "tlcg_state_bits": (C.c_int, [M]),
        "tlcg_init_count": (U64, [M]),
        "tlcg_create": (C.c_int, [M, O, C.POINTER(P)]),
        "tlcg_destroy": (None, [P]),
        "tlcg_last_error": (C.c_char_p, [P]),
        "tlcg_init": (C.c_int, [P, S]),
        "tlcg_step_level": (C.c_int, [P, S]),
        "tlcg_run": (C.c_int, [P, S]),
        "tlcg_level_sizes": (C.c_int, [P, C.POINTER(U64), I32, C.POINTER(I32)]),
        "tlcg_level_generated": (C.c_int, [P, C.POINTER(U64), I32, C.POINTER(I32)]),
        "tlcg_trace": (C.c_int, [P, C.POINTER(U64), C.POINTER(I32), I32, C.POINTER(I32)]),
        "tlcg_state_at": (C.c_int, [P, U64, C.POINTER(U64), C.POINTER(U64)]),
        "tlcg_copy_states": (C.c_int, [P, U64, U64, C.POINTER(U64)]),
        "tlcg_ordinal_bits": (C.c_int, [M]),
        "tlcg_action_of_ordinal": (C.c_int, [M, I32]),
        "tlcg_decode": (C.c_int, [M, U64, C.c_char_p, I32]),
        "tlcg_host_init_state": (U64, [M, U64]),
        "tlcg_host_successors": (C.c_int, [M, U64, C.POINTER(U64), C.POINTER(I32), I32]),
        "tlcg_host_check_invariants": (C.c_int, [M, U64]),
        "tlcg_host_component_selfcheck": (C.c_int64, [M, U64, U64]),
        "tlcg_host_tree_slot_probes": (C.c_int, [M, U64, C.POINTER(C.c_int64)]),
        "tlcg_host_termination_counterexample": (C.c_int64, [M]),
        "tlcg_owner": (C.c_int, [P, U64]),
        "tlcg_expand": (C.c_int, [P, S]),
        "tlcg_outbox": (C.c_int, [P, I32, C.POINTER(P), C.POINTER(U64)]),
        "tlcg_inbox": (C.c_int, [P, U64, C.POINTER(P)]),
        "tlcg_absorb": (C.c_int, [P, U64, S]),
        "tlcg_end_level": (C.c_int, [P, S]),
        "tlcg_outbox_read": (C.c_int, [P, I32, P, U64]),
        "tlcg_outbox_gather": (C.c_int, [P, P]),
        "tlcg_state_words": (C.c_int, [M]),
        "tlcg_checkpoint": (C.c_int, [P, C.c_char_p]),
        "tlcg_recover": (C.c_int, [P, C.c_char_p, S]),
        "tlcg_decode_words": (C.c_int, [M, C.POINTER(U64), C.c_char_p, I32]),
        "tlcg_host_init_state_words": (C.c_int, [M, U64, C.POINTER(U64)]),
        "tlcg_host_successors_words": (C.c_int, [M, C.POINTER(U64), C.POINTER(U64), C.POINTER(I32), I32]),
        "tlcg_host_check_invariants_words": (C.c_int, [M, C.POINTER(U64)]),
        "tlcg_host_check_invariants_batch": (C.c_int, [M, C.POINTER(U64), U64, C.POINTER(I32)]),
        "tlcg_trace_words": (C.c_int, [P, C.POINTER(U64), C.POINTER(I32), I32, C.POINTER(I32)]),
        "tlcg_state_at_words": (C.c_int, [P, U64, C.POINTER(U64), C.POINTER(U64)]),
        "tlcg_copy_states_words": (C.c_int, [P, U64, U64, C.POINTER(U64)]),
        "tlcg_tlc_stop_stats": (C.c_int, [P, C.POINTER(U64), C.POINTER(U64), C.POINTER(U64)]),
        "tlcg_outdegree": (C.c_int, [P, C.POINTER(U64), I32, C.POINTER(I32)]),
        "tlcg_expansions": (C.c_int, [P, C.POINTER(U64)]),
        "tlcg_absorb_records": (C.c_int, [P, P, U64, S]),
        "tlcg_stream": (P, [P]),
        "tlcg_peer_access": (C.c_int, [I32]),
        "tlcg_device_count": (C.c_int, []),
        "tlcg_exchange_local": (C.c_int, [C.POINTER(P), I32, C.POINTER(U64)]),
        "tlcg_partition_closed": (C.c_int, [P]),
        "tlcg_run_node": (C.c_int, [M, O, I32, S, C.POINTER(U64), I32, C.POINTER(I32), C.c_char_p, I32]),
        "tlcg_run_node_trace": (C.c_int, [M, O, I32, S, C.POINTER(U64), I32, C.POINTER(I32), C.POINTER(U64),
                                          C.POINTER(I32), I32, C.POINTER(I32), C.c_char_p, I32]),
        "tlcg_node_create": (C.c_int, [M, O, I32, C.POINTER(P), C.c_char_p, I32]),
        "tlcg_node_run": (C.c_int, [P, S, C.POINTER(U64), I32, C.POINTER(I32), C.POINTER(U64), C.POINTER(I32), I32,
                                    C.POINTER(I32), C.c_char_p, I32]),
        "tlcg_node_destroy": (None, [P]),
        "tlcg_comm_available": (C.c_int, []),
        "tlcg_comm_unique_id": (C.c_int, [P, I32]),
        "tlcg_comm_init": (C.c_int, [P, P, I32]),
        "tlcg_comm_size": (C.c_int, [P]),
        "tlcg_run_comm": (C.c_int, [P, S, C.POINTER(U64), I32, C.POINTER(I32)]),
        "tlcg_check_termination": (C.c_int, [M, O, I32, C.POINTER(tlcg_liveness), C.POINTER(U64),
                                             C.POINTER(I32), I32, C.POINTER(I32), C.c_char_p, I32]),
        "tlcg_jit_selftest": (C.c_int, [M, C.c_char_p, I32, C.c_char_p, I32][:1] + [C.c_char_p, C.c_char_p, I32]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


@dataclass
class Model:
    """Constants of compaction.tla:10-18 as a TLC cfg binds them."""
    msg_sent_limit: int = 3          # MessageSentLimit
    compaction_times_limit: int = 3  # CompactionTimesLimit
    consume_times_limit: int = 2     # ConsumeTimesLimit
    max_crash_times: int = 1         # MaxCrashTimes
    model_consumer: bool = False     # ModelConsumer
    model_producer: bool = False     # ModelProducer
    retain_null_key: bool = True     # RetainNullKey
    key_space: Sequence[int] = (1, 2)
    value_space: Sequence[int] = (1, 2)
    invariants: Sequence[str] = ("TypeSafe", "CompactionHorizonCorrectness")
    check_deadlock: bool = True
    # definitions added to the module (BASELINE config 5): "Name" or
    # "Name(p1, p2)" -> TLA+ body text; INVARIANTS may name the zero-argument
    # ones (include/tlcgpu.h tlcg_model.user_defs).  A name here shadows the
    # spec's invariant of that name.
    user_defs: Optional[dict] = None

    def user_defs_text(self) -> Optional[str]:
        """tlcg_model.user_defs: a "@@DEF name params" header line per definition, then its body"""
        if not self.user_defs:
            return None
        out = []
        for head, body in self.user_defs.items():
            name, _, rest = head.partition("(")
            params = [p.strip() for p in rest.rstrip(")").split(",") if p.strip()]
            out.append("@@DEF " + " ".join([name.strip()] + params))
            out.append(body)
        return "\n".join(out) + "\n"

    def user_names(self) -> List[str]:
        return [h.partition("(")[0].strip() for h in (self.user_defs or {})]

    def to_c(self) -> tlcg_model:
        m = tlcg_model()
        m.msg_sent_limit = self.msg_sent_limit
        m.compaction_times_limit = self.compaction_times_limit
        m.consume_times_limit = self.consume_times_limit
        m.max_crash_times = self.max_crash_times
        m.model_consumer = int(bool(self.model_consumer))
        m.model_producer = int(bool(self.model_producer))
        m.retain_null_key = int(bool(self.retain_null_key))
        m.check_deadlock = int(bool(self.check_deadlock))
        if len(self.key_space) > MAX_SET or len(self.value_space) > MAX_SET:
            raise ValueError("KeySpace/ValueSpace larger than 63 elements")
        m.n_keys = len(self.key_space)
        m.n_values = len(self.value_space)
        for i, k in enumerate(self.key_space):
            m.keys[i] = int(k)
        for i, v in enumerate(self.value_space):
            m.values[i] = int(v)
        if len(self.invariants) > MAX_INV:
            raise ValueError("too many invariants")
        m.n_invariants = len(self.invariants)
        users = self.user_names()
        for i, name in enumerate(self.invariants):
            if name in users:
                m.invariants[i] = INV_USER + users.index(name)
            elif name in INVARIANTS:
                m.invariants[i] = INVARIANTS.index(name)
            else:
                raise ValueError(f"unknown invariant {name}")
        text = self.user_defs_text()
        if text is not None:
            m.user_defs = text.encode()  # (ctypes keeps the bytes alive with the struct)
        return m

    def oracle_args(self) -> List[str]:
        """Command-line of oracle/build/tlc_oracle for the same constants (tests only)."""
        return ["-N", str(self.msg_sent_limit), "-C", str(self.compaction_times_limit),
                "-K", str(self.max_crash_times), "-ctl", str(self.consume_times_limit),
                "-keys", ",".join(map(str, self.key_space)) or "", "-values",
                ",".join(map(str, self.value_space)) or "", "-retain", str(int(self.retain_null_key)),
                "-producer", str(int(self.model_producer)), "-consumer", str(int(self.model_consumer)),
                "-inv", ",".join(self.invariants)] + ([] if self.check_deadlock else ["-nodeadlock"])


def check_model(model: Model) -> Optional[str]:
    """ASSUME (compaction.tla:25-35) + packing; None if fine, else the message."""
    lib = load_library()
    buf = C.create_string_buffer(512)
    m = model.to_c()
    return None if lib.tlcg_check_model(C.byref(m), buf, 512) == 0 else buf.value.decode()


def state_bits(model: Model) -> int:
    m = model.to_c()
    return load_library().tlcg_state_bits(C.byref(m))


def init_count(model: Model) -> int:
    m = model.to_c()
    return load_library().tlcg_init_count(C.byref(m))


def state_words(model: Model) -> int:
    """uint64 words per packed state: 1 (<= 63 bits) or 2 (wide, <= 126 bits)."""
    m = model.to_c()
    return load_library().tlcg_state_words(C.byref(m))


def _to_words(state: int, w: int):
    return (C.c_uint64 * w)(*[(state >> (64 * i)) & 0xFFFFFFFFFFFFFFFF for i in range(w)])


def _from_words(buf, i: int, w: int) -> int:
    return sum(int(buf[i * w + k]) << (64 * k) for k in range(w))


def decode(model: Model, state: int) -> str:
    """TLC value syntax of a packed state (a Python int of either width)."""
    lib = load_library()
    m = model.to_c()
    buf = C.create_string_buffer(1 << 16)
    n = lib.tlcg_decode_words(C.byref(m), _to_words(state, state_words(model)), buf, len(buf))
    if n < 0:
        raise ValueError("bad model")
    return buf.value.decode()


def host_init_state(model: Model, idx: int) -> int:
    m = model.to_c()
    w = state_words(model)
    out = (C.c_uint64 * 2)()
    if load_library().tlcg_host_init_state_words(C.byref(m), idx, out) != 0:
        raise ValueError("bad model")
    return _from_words(out, 0, w)


def host_successors(model: Model, state: int) -> List[Tuple[str, int]]:
    lib = load_library()
    m = model.to_c()
    w = state_words(model)
    cap = 8192
    out = (C.c_uint64 * (cap * w))()
    acts = (C.c_int32 * cap)()
    n = lib.tlcg_host_successors_words(C.byref(m), _to_words(state, w), out, acts, cap)
    if n < 0:
        raise RuntimeError("evaluation error")
    return [(ACTIONS[acts[i]], _from_words(out, i, w)) for i in range(n)]


def host_component_selfcheck(model: Model, first: int, n: int) -> int:
    """States on which the component engine's specialized evaluators were
    compared with the generic ones (< 0: a disagreement)."""
    m = model.to_c()
    return load_library().tlcg_host_component_selfcheck(C.byref(m), C.c_uint64(first), C.c_uint64(n))


def host_tree_slot_probes(model: Model, comp: int):
    """(insert calls, probe trips with the displacement table, without it) of
    the closed tree's FPSet on component `comp`, replayed on the host; None
    when the closed tree does not take it."""
    m = model.to_c()
    out = (C.c_int64 * 3)()
    r = load_library().tlcg_host_tree_slot_probes(C.byref(m), C.c_uint64(comp), out)
    if r == -2:
        raise ValueError("bad model")
    return None if r < 0 else (out[0], out[1], out[2])


def host_check_invariants_batch(model: Model, states: Sequence[int]) -> List[int]:
    """check_invariants of every state (-1: all hold, else index << 1 | is_error), one model build"""
    m = model.to_c()
    w = state_words(model)
    buf = (C.c_uint64 * (len(states) * w))()
    for i, s in enumerate(states):
        for k in range(w):
            buf[i * w + k] = (s >> (64 * k)) & 0xFFFFFFFFFFFFFFFF
    out = (C.c_int32 * max(1, len(states)))()
    if load_library().tlcg_host_check_invariants_batch(C.byref(m), buf, len(states), out) != 0:
        raise ValueError(check_model(model) or "bad model")
    return list(out)[:len(states)]


def host_check_invariants(model: Model, state: int) -> int:
    m = model.to_c()
    return load_library().tlcg_host_check_invariants_words(C.byref(m), _to_words(state, state_words(model)))


@dataclass
class Liveness:
    """PROPERTY Termination (compaction.tla:303-307) checked on the GPU."""
    holds: bool
    kind: str                    # "holds", "stuttering" or "cycle"
    fairness: str                # "none" (Spec) or "wf" (Spec /\ WF_vars(Next))
    depth: int                   # BFS levels of G' (the not-P part of the graph)
    states_notp: int
    init_notp: int
    edges_notp: int
    stuck: int
    on_cycles: int
    peel_rounds: int
    trace: List[Tuple[str, int]] = field(default_factory=list)  # (action into it, state)
    loop_to: int = -1            # -1: the counterexample ends stuttering
    back_action: Optional[str] = None
    kernel_ms: float = 0.0
    wall_ms: float = 0.0


def check_termination(model: Model, fairness: str = "none", device: int = 0, state_capacity: int = 0,
                      log2_fpset_slots: int = 0) -> Liveness:
    r"""TLC's liveness check of PROPERTY Termination under Spec (fairness
    "none") or Spec /\ WF_vars(Next) ("wf"), through tlcg_check_termination."""
    lib = load_library()
    m = model.to_c()
    o = tlcg_opts()
    o.device, o.state_capacity, o.log2_fpset_slots = device, state_capacity, log2_fpset_slots
    out = tlcg_liveness()
    w = state_words(model)
    cap = 1 << 12
    states = (C.c_uint64 * (cap * w))()
    acts = (C.c_int32 * cap)()
    n = C.c_int32(0)
    err = C.create_string_buffer(512)
    rc = lib.tlcg_check_termination(C.byref(m), C.byref(o), FAIRNESS[fairness], C.byref(out), states, acts, cap,
                                    C.byref(n), err, len(err))
    if rc != 0:
        raise RuntimeError(f"tlcg_check_termination: {rc}: {err.value.decode()}")
    trace = [("Init" if acts[i] < 0 else ACTIONS[acts[i]], _from_words(states, i, w)) for i in range(n.value)]
    return Liveness(bool(out.holds), LIVE_KINDS[out.kind], fairness, out.depth, out.states_notp, out.init_notp,
                    out.edges_notp, out.stuck, out.on_cycles, out.peel_rounds, trace, out.loop_to,
                    ACTIONS[out.back_action] if out.loop_to >= 0 else None, out.kernel_ms, out.wall_ms)


@dataclass
class Result:
    status: str
    generated: int
    distinct: int
    depth: int
    left_on_queue: int
    levels: List[int] = field(default_factory=list)
    invariant: Optional[str] = None
    action: Optional[str] = None
    collision_optimistic: float = 0.0
    kernel_ms: float = 0.0
    expand_ms: float = 0.0
    levels_redone: int = 0
    engine: str = ""
    host_states: int = 0
    fpset_host_states: int = 0
    trace: List[Tuple[str, int]] = field(default_factory=list)
    transport: str = ""  # multi-rank runs: "local" (threads, device copies) or "rccl"
    tlc_exact: bool = False  # an error whose trace and tlc_stop_stats() are TLC -workers 1's (tlcg_stats.tlc_exact)
    jit_used: int = 0  # tlcg_stats.jit_used: which specialized kernels ran (include/tlcgpu.h)


class Checker:
    """One checking context on one GPU (libtlcgpu tlcg_ctx)."""

    def __init__(self, model: Model, device: int = 0, log2_fpset_slots: int = 0, state_capacity: int = 0,
                 tlc_order: bool = False, rank: int = 0, world: int = 1, partition: int = 0,
                 engine: str = "auto", spill: bool = False, device_store_cap: int = 0,
                 fpset_spill: bool = False, log2_fpset_max: int = 0, outdegree: bool = False):
        self.lib = load_library()
        self.model = model
        self._m = model.to_c()
        o = tlcg_opts()
        o.device, o.log2_fpset_slots, o.state_capacity = device, log2_fpset_slots, state_capacity
        o.tlc_order, o.rank, o.world, o.partition = int(tlc_order), rank, world, partition
        o.engine = ENGINES[engine]
        o.spill, o.device_store_cap = int(spill), device_store_cap
        o.fpset_spill, o.log2_fpset_max = int(fpset_spill), log2_fpset_max
        o.outdegree = int(outdegree)
        self._o = o
        self.ctx = C.c_void_p()
        rc = self.lib.tlcg_create(C.byref(self._m), C.byref(o), C.byref(self.ctx))
        if rc != 0:
            msg = self.lib.tlcg_last_error(self.ctx).decode() if self.ctx else "tlcg_create failed"
            self.close()
            raise RuntimeError(f"tlcg_create: {msg} ({rc})")
        self.stats = tlcg_stats()
        self.words = state_words(model)

    def close(self):
        if getattr(self, "ctx", None):
            self.lib.tlcg_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _chk(self, rc: int, what: str):
        if rc != 0:
            raise RuntimeError(f"{what}: {self.lib.tlcg_last_error(self.ctx).decode()} ({rc})")

    def init(self):
        self._chk(self.lib.tlcg_init(self.ctx, C.byref(self.stats)), "tlcg_init")
        return self.stats

    def step_level(self):
        self._chk(self.lib.tlcg_step_level(self.ctx, C.byref(self.stats)), "tlcg_step_level")
        return self.stats

    def run_raw(self):
        """tlcg_run only (no host work after it): for timing."""
        self._chk(self.lib.tlcg_run(self.ctx, C.byref(self.stats)), "tlcg_run")
        return self.stats

    def checkpoint(self, path: str):
        """TLC -checkpoint: the committed levels to `path` (global engine, between levels)."""
        self._chk(self.lib.tlcg_checkpoint(self.ctx, path.encode()), "tlcg_checkpoint")

    def recover(self, path: str):
        """TLC -recover: resume from `path`; continue with step_level()."""
        self._chk(self.lib.tlcg_recover(self.ctx, path.encode(), C.byref(self.stats)), "tlcg_recover")
        return self.stats

    def level_sizes(self) -> List[int]:
        buf = (C.c_uint64 * 65536)()
        n = C.c_int32()
        self._chk(self.lib.tlcg_level_sizes(self.ctx, buf, 65536, C.byref(n)), "tlcg_level_sizes")
        return [buf[i] for i in range(min(n.value, 65536))]

    def level_generated(self) -> List[int]:
        """[0] initial states, [k] successors generated by expanding level k - 1
        (tlcg_level_generated)."""
        buf = (C.c_uint64 * 65536)()
        n = C.c_int32()
        self._chk(self.lib.tlcg_level_generated(self.ctx, buf, 65536, C.byref(n)), "tlcg_level_generated")
        return [buf[i] for i in range(min(n.value, 65536))]

    def trace(self) -> List[Tuple[str, int]]:
        cap, w = 1 << 16, self.words
        st = (C.c_uint64 * (cap * w))()
        ac = (C.c_int32 * cap)()
        n = C.c_int32()
        self._chk(self.lib.tlcg_trace_words(self.ctx, st, ac, cap, C.byref(n)), "tlcg_trace_words")
        return [("Init" if ac[i] < 0 else ACTIONS[ac[i]], _from_words(st, i, w)) for i in range(n.value)]

    def copy_states(self, first: int, n: int) -> List[int]:
        w = self.words
        buf = (C.c_uint64 * (max(n, 1) * w))()
        self._chk(self.lib.tlcg_copy_states_words(self.ctx, first, n, buf), "tlcg_copy_states_words")
        return [_from_words(buf, i, w) for i in range(n)]

    def tlc_stop_stats(self) -> Tuple[int, int, int]:
        """(generated, distinct, left on queue) where a one-worker TLC run stops on
        this error (tlcg_tlc_stop_stats; global engine, TLC order)."""
        g, d, q = C.c_uint64(), C.c_uint64(), C.c_uint64()
        self._chk(self.lib.tlcg_tlc_stop_stats(self.ctx, C.byref(g), C.byref(d), C.byref(q)), "tlcg_tlc_stop_stats")
        return g.value, d.value, q.value

    def expansions(self) -> int:
        """state expansions the last check's kernels made (tlcg_expansions):
        distinct / expansions is 1 for a per-state kernel, the components per
        walk for the one-walk-per-wavefront kernel"""
        n = C.c_uint64()
        self._chk(self.lib.tlcg_expansions(self.ctx, C.byref(n)), "tlcg_expansions")
        return n.value

    def outdegree(self) -> List[int]:
        """TLC's outdegree histogram of the completed check (tlcg_outdegree):
        [k] = states whose expansion discovered k new states."""
        buf = (C.c_uint64 * 4100)()
        n = C.c_int32()
        self._chk(self.lib.tlcg_outdegree(self.ctx, buf, 4100, C.byref(n)), "tlcg_outdegree")
        return [buf[i] for i in range(n.value)]

    def state_at(self, gidx: int) -> Tuple[int, int]:
        s, p = (C.c_uint64 * 2)(), C.c_uint64()
        self._chk(self.lib.tlcg_state_at_words(self.ctx, gidx, s, C.byref(p)), "tlcg_state_at_words")
        return _from_words(s, 0, self.words), p.value

    def result(self, with_trace: bool = True) -> Result:
        s = self.stats
        status = STATUS[s.status]
        r = Result(status=status, generated=s.generated, distinct=s.distinct, depth=s.depth,
                   left_on_queue=0 if status == "ok" else s.frontier, levels=self.level_sizes(),
                   collision_optimistic=s.fp_collision_optimistic, kernel_ms=s.kernel_ms,
                   expand_ms=s.expand_ms, levels_redone=s.levels_redone,
                   engine={v: k for k, v in ENGINES.items()}.get(s.engine, "?"), host_states=s.host_states,
                   fpset_host_states=s.fpset_host_states, tlc_exact=bool(s.tlc_exact), jit_used=s.jit_used)
        if s.invariant >= 0:
            r.invariant = self.model.invariants[s.invariant]
        if s.action >= 0:
            r.action = ACTIONS[s.action]
        if with_trace and status not in ("ok", "running"):
            r.trace = self.trace()
        return r

    def run(self, with_trace: bool = True) -> Result:
        self.run_raw()
        return self.result(with_trace)


def run(model: Model, **kw) -> Result:
    """Convenience: check `model` on one GPU."""
    ck = Checker(model, **kw)
    try:
        return ck.run()
    finally:
        ck.close()


def _node_opts(device=0, log2_fpset_slots=0, state_capacity=0, partition=0, engine="auto", spill=False,
               device_store_cap=0, fpset_spill=False, log2_fpset_max=0):
    o = tlcg_opts()
    o.device, o.log2_fpset_slots, o.state_capacity, o.partition = device, log2_fpset_slots, state_capacity, partition
    o.engine = ENGINES[engine]
    o.spill, o.device_store_cap = int(spill), device_store_cap
    o.fpset_spill, o.log2_fpset_max = int(fpset_spill), log2_fpset_max
    return o


class Node:
    """The ranks of one node kept across checks (tlcg_node_create / run /
    destroy): rank r on device r mod device_count, driven by one host thread
    each; the contexts (FPSet shards, stores, outboxes) and the transport are
    built once, so run() costs the level loop only.  run() returns what
    run_node returns."""

    def __init__(self, model: Model, ranks: int, **opts):
        self.lib = load_library()
        self.model = model
        self._m = model.to_c()  # (kept alive: the contexts copy it, user_defs included)
        self.node = C.c_void_p()
        err = C.create_string_buffer(1024)
        rc = self.lib.tlcg_node_create(C.byref(self._m), C.byref(_node_opts(**opts)), ranks, C.byref(self.node),
                                       err, 1024)
        if rc != 0:
            raise RuntimeError(f"tlcg_node_create: {err.value.decode()} ({rc})")

    def run(self) -> Result:
        model, lib = self.model, self.lib
        st = tlcg_stats()
        lv = (C.c_uint64 * 65536)()
        n = C.c_int32()
        err = C.create_string_buffer(1024)
        w = state_words(model)
        tcap = 4096
        tst = (C.c_uint64 * (tcap * w))()
        tact = (C.c_int32 * tcap)()
        tlen = C.c_int32()
        rc = lib.tlcg_node_run(self.node, C.byref(st), lv, 65536, C.byref(n), tst, tact, tcap, C.byref(tlen), err, 1024)
        if rc != 0:
            raise RuntimeError(f"tlcg_node_run: {err.value.decode()} ({rc})")
        status = STATUS[st.status]
        r = Result(status=status, generated=st.generated, distinct=st.distinct, depth=st.depth,
                   left_on_queue=0 if status == "ok" else st.frontier, levels=[lv[i] for i in range(n.value)],
                   collision_optimistic=st.fp_collision_optimistic, kernel_ms=st.kernel_ms, expand_ms=st.expand_ms,
                   levels_redone=st.levels_redone, engine={v: k for k, v in ENGINES.items()}.get(st.engine, "?"),
                   host_states=st.host_states, fpset_host_states=st.fpset_host_states,
                   transport={1: "local", 2: "rccl"}.get(st.transport, ""))
        if st.invariant >= 0:
            r.invariant = model.invariants[st.invariant]
        if st.action >= 0:
            r.action = ACTIONS[st.action]
        r.trace = [("Init" if tact[i] < 0 else ACTIONS[tact[i]], _from_words(tst, i, w))
                   for i in range(min(tlen.value, tcap))]
        return r

    def close(self):
        if self.node:
            self.lib.tlcg_node_destroy(self.node)
            self.node = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001  (interpreter shutdown)
            pass


def run_node(model: Model, ranks: int, device: int = 0, log2_fpset_slots: int = 0, state_capacity: int = 0,
             partition: int = 0, engine: str = "auto", spill: bool = False, device_store_cap: int = 0,
             fpset_spill: bool = False, log2_fpset_max: int = 0) -> Result:
    """The check by this one process on `ranks` contexts, rank r on device
    r mod device_count (tlcg_node_create + tlcg_node_run; `tlc-hip -gpus N`).
    On an error .trace is the counterexample walked across the ranks' stores
    (a shortest one; TLC -workers 1's own trace: Checker(..., tlc_order=True))."""
    node = Node(model, ranks, device=device, log2_fpset_slots=log2_fpset_slots, state_capacity=state_capacity,
                partition=partition, engine=engine, spill=spill, device_store_cap=device_store_cap,
                fpset_spill=fpset_spill, log2_fpset_max=log2_fpset_max)
    try:
        return node.run()
    finally:
        node.close()
