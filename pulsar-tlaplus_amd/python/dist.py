"""Multi-GPU BFS: one process (rank) per MI355X, FPSet hash-partitioned by owner.

This is the distributed counterpart of TLC's FPSetManager (tlc2.tool.fp,
fingerprint-partitioned FPSet): every rank owns the states whose owner hash
(mix64 of the partition key) maps to it.

Two regimes, chosen by libtlcgpu from the model:

* closed partition -- with ModelProducer = FALSE no action writes `messages`
  (compaction.tla:87,100,132,139,145,151,165,182,186,214), so keying the owner
  hash on `messages` keeps every successor on its parent's rank.  Each rank
  runs its BFS to completion with no data-path collective; one all-reduce
  combines the counts (distinct/generated sum, depth max, first error).
* open partition -- otherwise (Producer appends to `messages`) each level is
  expand -> all-to-all of 16-byte {state, parent_ref} records to their owners
  (RCCL over xGMI with the nccl backend) -> absorb -> all-reduce of the level
  counters to decide termination.

`Engine` is the per-rank face of include/tlcgpu.h's partitioned API; the GPU
engine wraps libtlcgpu, the tests plug a CPU stand-in into the same driver.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from typing import List, Optional, Tuple

import torch
import torch.distributed as dist

import tlcgpu

STATUS_RUNNING, STATUS_DONE = 0, 1


@dataclass
class DistResult:
    status: str
    generated: int
    distinct: int
    depth: int
    levels: List[int]
    kernel_ms: float
    expand_ms: float
    closed: bool
    invariant: Optional[int] = None         # index into the model's invariants (first error)
    first_error_rank: Optional[int] = None
    engine: str = ""                         # "tree": the ranks ran shares of the component tree
    trace: List[Tuple[str, int]] = field(default_factory=list)  # run_native: walked across the ranks' stores


class GpuEngine:
    """One rank's libtlcgpu context (the partitioned C-ABI)."""

    def __init__(self, model: tlcgpu.Model, rank: int, world: int, device: int, **opts):
        self.model, self.opts = model, dict(opts)
        self.ck = tlcgpu.Checker(model, device=device, rank=rank, world=world, **opts)
        self.lib, self.ctx, self.stats = self.ck.lib, self.ck.ctx, self.ck.stats
        self.world, self.rank, self.device = world, rank, device
        self.closed = world == 1 or (not model.model_producer and opts.get("partition", 0) in (0, 1))

    def reopen_global(self):
        """a new context on the global engine (the ranks left the component tree)"""
        self.ck.close()
        self.ck = tlcgpu.Checker(self.model, device=self.device, rank=self.rank, world=self.world,
                                 **dict(self.opts, engine="global"))
        self.lib, self.ctx, self.stats = self.ck.lib, self.ck.ctx, self.ck.stats

    def run_closed(self) -> tlcgpu.tlcg_stats:
        return self.ck.run_raw()

    def init(self):
        return self.ck.init()

    def expand(self) -> List[int]:
        self.ck._chk(self.lib.tlcg_expand(self.ctx, C.byref(self.stats)), "tlcg_expand")
        counts = []
        for dst in range(self.world):
            p, n = C.c_void_p(), C.c_uint64()
            self.lib.tlcg_outbox(self.ctx, dst, C.byref(p), C.byref(n))
            counts.append(n.value)
        return counts

    def outbox(self, dst: int) -> torch.Tensor:
        """This rank's records for `dst`, copied (in stream order) to a new tensor."""
        p, n = C.c_void_p(), C.c_uint64()
        self.lib.tlcg_outbox(self.ctx, dst, C.byref(p), C.byref(n))
        t = torch.empty((n.value, 2), dtype=torch.int64, device=f"cuda:{self.device}")
        torch.cuda.synchronize(self.device)
        if n.value:
            self.ck._chk(self.lib.tlcg_outbox_read(self.ctx, dst, C.c_void_p(t.data_ptr()), n.value),
                         "tlcg_outbox_read")
        return t

    def outbox_all(self, counts: List[int], device) -> torch.Tensor:
        """Every destination's records, destination-major (the all-to-all send
        buffer), gathered by the library with one stream synchronization."""
        t = torch.empty((sum(counts), 2), dtype=torch.int64, device=device)
        if t.shape[0]:
            if t.device.type == "cuda":
                torch.cuda.synchronize(self.device)
            self.ck._chk(self.lib.tlcg_outbox_gather(self.ctx, C.c_void_p(t.data_ptr())), "tlcg_outbox_gather")
        return t

    def absorb(self, recs: torch.Tensor):
        """Insert records from other ranks (device or host tensor, [n, 2] int64)."""
        recs = recs.contiguous()
        if recs.device.type == "cuda":
            torch.cuda.synchronize(self.device)  # torch's producer of `recs` is done
        self.ck._chk(self.lib.tlcg_absorb_records(self.ctx, C.c_void_p(recs.data_ptr()), recs.shape[0],
                                                  C.byref(self.stats)), "tlcg_absorb_records")

    def end_level(self):
        self.ck._chk(self.lib.tlcg_end_level(self.ctx, C.byref(self.stats)), "tlcg_end_level")
        return self.stats

    def level_sizes(self) -> List[int]:
        return self.ck.level_sizes()

    def level_generated(self) -> List[int]:
        return self.ck.level_generated()

    def new_tensor(self, shape, dtype):
        return torch.empty(shape, dtype=dtype, device=f"cuda:{self.device}")

    def close(self):
        self.ck.close()


def _reduce_result(engine, stats, group, dev: torch.device) -> DistResult:
    """Combine the ranks' results like one context's level loop would report
    them.  The first error -- lowest level, then lowest rank (node.cpp does
    the same) -- gives the verdict and the depth E + 1.  A closed partition's
    ranks run on independently past another rank's error, so every rank's
    counts are cut at the end of level E: levels 0..E, and the states
    generated up to that level (tlcg_level_generated)."""
    levels = engine.level_sizes()
    lgen = engine.level_generated()
    me = dist.get_rank(group)
    st = int(stats.status)
    none = 1 << 62
    key = torch.tensor([(len(levels) << 16) | me if st >= 2 else none], dtype=torch.int64, device=dev)
    dist.all_reduce(key, op=dist.ReduceOp.MIN, group=group)
    k = int(key.item())
    first, cut = (None, None) if k == none else (k & 0xFFFF, k >> 16)
    mine = levels if cut is None else levels[:cut]
    g = sum(lgen) if cut is None else sum(lgen[:cut])
    inv = getattr(stats, "invariant", -1)
    info = torch.tensor([len(mine), g, st if first == me else 0, inv + 1 if first == me else 0],
                        dtype=torch.int64, device=dev)
    n = torch.tensor([len(mine)], dtype=torch.int64, device=dev)
    dist.all_reduce(n, op=dist.ReduceOp.MAX, group=group)
    lv = torch.zeros(max(int(n.item()), 1), dtype=torch.int64, device=dev)
    if mine:
        lv[: len(mine)] = torch.tensor(mine, dtype=torch.int64, device=dev)
    dist.all_reduce(lv, op=dist.ReduceOp.SUM, group=group)
    dist.all_reduce(info, op=dist.ReduceOp.SUM, group=group)
    levels_all = [int(x) for x in lv.tolist()]
    while levels_all and levels_all[-1] == 0:
        levels_all.pop()
    code, inv_all = int(info[2].item()), int(info[3].item()) - 1
    return DistResult(status=tlcgpu.STATUS[code] if first is not None else "ok", generated=int(info[1].item()),
                      distinct=sum(levels_all), depth=cut if cut is not None else len(levels_all),
                      levels=levels_all, kernel_ms=stats.kernel_ms, expand_ms=stats.expand_ms, closed=engine.closed,
                      invariant=inv_all if inv_all >= 0 else None, first_error_rank=first)


def init_native(engine: "GpuEngine", group=None) -> None:
    """An RCCL communicator inside libtlcgpu for this rank (tlcg_comm_init):
    rank 0 makes the id, the group broadcasts it."""
    lib = engine.lib
    buf = C.create_string_buffer(128)
    obj = [b""]
    if dist.get_rank(group) == 0 and lib.tlcg_comm_unique_id(buf, 128) == 128:
        obj = [buf.raw]
    dist.broadcast_object_list(obj, src=0, group=group)  # (an empty id: every rank raises below)
    if len(obj[0]) != 128:
        raise RuntimeError(f"tlcg_comm_unique_id failed on rank 0 (RCCL available here: {lib.tlcg_comm_available()})")
    buf = C.create_string_buffer(obj[0], 128)
    engine.ck._chk(lib.tlcg_comm_init(engine.ctx, buf, 128), "tlcg_comm_init")


def run_native(engine: "GpuEngine") -> DistResult:
    """The whole check inside libtlcgpu (tlcg_run_comm): the level loop and its
    exchange run in C++ over RCCL -- all-gather of the per-destination counts,
    grouped send/recv of the records on the context's stream, all-reduce for
    termination and the combined result -- with no Python in the level loop.
    init_native() first."""
    lib = engine.lib
    st = tlcgpu.tlcg_stats()
    lv = (C.c_uint64 * 65536)()
    n = C.c_int32()
    engine.ck._chk(lib.tlcg_run_comm(engine.ctx, C.byref(st), lv, 65536, C.byref(n)), "tlcg_run_comm")
    levels = [lv[i] for i in range(n.value)]
    trace = []
    if st.status >= 2:  # an error: the counterexample walked across the ranks' stores (every rank holds it)
        trace = engine.ck.trace()
    return DistResult(status=tlcgpu.STATUS[st.status], generated=st.generated, distinct=st.distinct, depth=st.depth,
                      levels=levels, kernel_ms=st.kernel_ms, expand_ms=st.expand_ms, closed=engine.closed,
                      invariant=st.invariant if st.invariant >= 0 else None,
                      engine=tlcgpu.ENGINE_NAMES.get(int(st.engine), "?"), trace=trace)


def _transport_device(group, dev: torch.device) -> torch.device:
    """Where exchanged records live: on the GPU for RCCL (nccl backend, xGMI),
    in host memory for gloo (rehearsals of the same level loop)."""
    return dev if dist.get_backend(group) == "nccl" else torch.device("cpu")


def run(engine, group=None, dev: Optional[torch.device] = None, timing: Optional[dict] = None) -> DistResult:
    """Model-check with every rank of `group` (engine = this rank's share).

    `timing`, when given, accumulates the seconds spent in the exchange
    (outbox gather, the two all-to-alls, inbox copy) under "exchange_s"."""
    import time
    dev = dev or torch.device("cpu")
    world = dist.get_world_size(group)
    if engine.closed:
        stats = engine.run_closed()
        return _reduce_result(engine, stats, group, dev)
    xdev = _transport_device(group, dev)
    stats = engine.init()
    # Producer modelled: each rank ran its subtrees of the component tree in
    # init (csrc/tree.h, no exchange) -- unless one of them handed the model
    # to the global engine (an error to report); then every rank does
    if hasattr(engine, "reopen_global"):
        tree = torch.tensor([1 if int(stats.engine) == 3 else 0], dtype=torch.int64, device=dev)
        dist.all_reduce(tree, op=dist.ReduceOp.SUM, group=group)
        if int(tree.item()) == world:
            r = _reduce_result(engine, stats, group, dev)
            r.engine = "tree"
            return r
        if int(stats.engine) == 3:
            engine.reopen_global()
            stats = engine.init()
    me = dist.get_rank(group)
    lv0 = engine.level_sizes()
    flags = torch.tensor([lv0[-1] if lv0 else 0, 1 if stats.status >= 2 else 0], dtype=torch.int64, device=dev)
    dist.all_reduce(flags, op=dist.ReduceOp.SUM, group=group)
    xs = 0.0
    while not flags[1].item() and flags[0].item():
        counts = engine.expand()
        t0 = time.perf_counter()
        # all-to-all: counts, then the records (16 bytes each), destination-major
        send_counts = torch.tensor(counts, dtype=torch.int64, device=xdev)
        send_counts[me] = 0
        recv_counts = torch.empty(world, dtype=torch.int64, device=xdev)
        dist.all_to_all_single(recv_counts, send_counts, group=group)
        rc = [int(x) for x in recv_counts.tolist()]
        sc = [int(x) for x in send_counts.tolist()]
        if hasattr(engine, "outbox_all"):
            send = engine.outbox_all(sc, xdev)
        else:  # per-destination stand-in engines (tests)
            send = torch.cat([engine.outbox(d) if sc[d] else torch.empty((0, 2), dtype=torch.int64)
                              for d in range(world)], 0).to(xdev)
        recv = torch.empty((sum(rc), 2), dtype=torch.int64, device=xdev)
        dist.all_to_all_single(recv, send, output_split_sizes=rc, input_split_sizes=sc, group=group)
        xs += time.perf_counter() - t0
        if recv.shape[0]:
            engine.absorb(recv)
        stats = engine.end_level()
        # global termination: any error, or no new state anywhere
        lv = engine.level_sizes()
        flags = torch.tensor([lv[-1] if lv else 0, 1 if stats.status >= 2 else 0], dtype=torch.int64, device=dev)
        dist.all_reduce(flags, op=dist.ReduceOp.SUM, group=group)
    if timing is not None:
        timing["exchange_s"] = timing.get("exchange_s", 0.0) + xs
    return _reduce_result(engine, stats, group, dev)
