"""Benchmark: distinct states/s of the BFS safety check of compaction.tla on the
scaled cfg (BASELINE.json metric), on 1..8 MI355X.

A step = one complete model check of the G9 config (SURVEY 8(d):
KeySpace = ValueSpace = {1..15}, MessageSentLimit = 3, CompactionTimesLimit = 3,
MaxCrashTimes = 1, RetainNullKey, no producer/consumer -> 1,040,187,392
distinct states, 1,392,508,928 generated, depth 20): FPSet cleared, Init,
then every BFS level until the queue is empty.  Inputs are the constants;
everything lives in HBM.

The headline (`value`, `ms_per_step`, `roofline`) is the fastest engine whose
timed kernel expands every distinct state: the on-chip engines' per-lane
kernels (each lane runs its own component's BFS: successors, FPSet probes,
invariants, store record per state), priced on SURVEY 8(d)'s 34.7 B per
distinct state.  Beside it: the HBM-FPSet engine (engines.global_hbm_fpset)
and the one-walk-per-wavefront kernels (engines.wave_quotient), which expand a
code graph once for M x 64 components -- a product quotient, no roofline.
With N GPUs the same job is split across N ranks
(strong scaling): without a Producer each rank runs a contiguous range of the
components (no data-path collective); the FPSet hash-partitioned by owner
with the per-level exchange (BASELINE config 4) is measured beside it, and a
producer-modelled cfg splits the component tree by subtrees.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config g9|m8|s|g9deep|p8]
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "pulsar-tlaplus_amd", "python"))

CONFIGS = {
    "g9": dict(keys=15, distinct=1_040_187_392, generated=1_392_508_928, depth=20),
    "m8": dict(keys=10, distinct=109_836_782, generated=147_039_563, depth=20),
    "s": dict(keys=2, distinct=45_198, generated=60_507, depth=20),
    # CompactionTimesLimit = 12, a 93-bit (two-word) state
    "g9deep": dict(keys=10, C=12, distinct=986_759_477, generated=1_119_626_552, depth=74),
    # an open state space: the producer modelled (the component tree on one
    # GPU; at N > 1 every level crosses ranks), oracle-pinned in tests/golden/p8.json
    "p8": dict(keys=7, producer=True, retain=False, distinct=91_781_506, generated=161_341_378, depth=23),
    # BASELINE config 5 at scale: G9 with an invariant the user adds to the
    # module (it holds, so the whole space is checked): the cfg's two spec
    # invariants plus LatestIsLast, compiled from its TLA+ text (user_inv.cpp)
    "g9u": dict(keys=15, distinct=1_040_187_392, generated=1_392_508_928, depth=20, user="LatestIsLast"),
    # the same with every invariant of tests/golden/user_inv.json's U_all_hold
    "g9uall": dict(keys=15, distinct=1_040_187_392, generated=1_392_508_928, depth=20,
                   user=("PhaseKnown", "LatestIsLast", "LedgerSorted", "KeysKnown", "MessageRec", "HeadFirst")),
}
# (and one config per user invariant alone: g9u_PhaseKnown, ...)
for _n in ("PhaseKnown", "LatestIsLast", "LedgerSorted", "KeysKnown", "MessageRec", "HeadFirst"):
    CONFIGS["g9u_" + _n] = dict(CONFIGS["g9"], user=_n)
# user invariants the g9u* configs add to compaction.tla (definitions by name;
# KeySet, ValueSet and NullKey are the module's own, restated for the library)
USER_DEFS = {
    "NullKey": "0",
    "KeySet": "KeySpace \\cup {NullKey}",
    "ValueSet": "ValueSpace \\cup {0}",
    "PhaseKnown": "compactorState \\in {Compactor_In_PhaseOne, Compactor_In_PhaseTwoWrite,\n"
                  "                   Compactor_In_PhaseTwoUpdateContext, Compactor_In_PhaseTwoUpdateHorizon,\n"
                  "                   Compactor_In_PhaseTwoPersistCusror, Compactor_In_PhaseTwoDeleteLedger}",
    "LatestIsLast": "phaseOneResult # Nil =>\n"
                    "  \\A k \\in DOMAIN phaseOneResult.latestForKey :\n"
                    "    /\\ messages[phaseOneResult.latestForKey[k]].key = k\n"
                    "    /\\ \\A i \\in 1..phaseOneResult.readPosition :\n"
                    "         messages[i].key = k => i <= phaseOneResult.latestForKey[k]",
    "LedgerSorted": "\\A l \\in 1..CompactionTimesLimit :\n"
                    "  compactedLedgers[l] # Nil =>\n"
                    "    \\A a \\in 1..Len(compactedLedgers[l]) : \\A b \\in 1..Len(compactedLedgers[l]) :\n"
                    "      a < b => compactedLedgers[l][a].id < compactedLedgers[l][b].id",
    "KeysKnown": "\\A i \\in 1..Len(messages) : messages[i].key \\in KeySet /\\ messages[i].value \\in ValueSet",
    "MessageRec": "\\A i \\in 1..Len(messages) :\n"
                  "   messages[i] = [id |-> i, key |-> messages[i].key, value |-> messages[i].value]",
    "HeadFirst": "Len(messages) > 0 => Head(messages).id = 1",
}
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
# algorithmic bytes per distinct state of the fused expand kernel:
# read the parent word (8 B) + write the new word and its parent entry (16 B)
# + one 8-B FPSet slot probe per non-stuttering successor (g'/d of them)
BYTES_PER_STATE_WORD = 8


# the newest round's profile of each kind (profiles/rNN_*), measured on the same kernels
PMC_PROFILE = "pmc_k_expand.json"
COMPONENT_BYTES_PER_STATE = 4  # the per-lane code pass writes one 32-bit record per state (component.h comp_record)
# the wave kernels (component_wave.h, tree_wave.h) walk a code graph once for
# M x 64 components (component.h WAVE_M / WAVE_M_USER / WAVE_M_BIG, tree.h TREE_WAVE_M)
WAVE_M, WAVE_M_USER, TREE_WAVE_M = 10, 4, 10
WAVE_M_BIG, WAVE_BIG_COMPS = 16, 1 << 23  # (component.h: models with many components)
# the per-state kernels of the on-chip engines: the one-walk-per-wavefront
# kernels off (the library's A/B switches)
PER_STATE_ENV = {"TLCG_COMP_WAVE": "0", "TLCG_TREE_WAVE": "0"}


class per_state_kernels:
    """the on-chip engines' per-lane kernels for the enclosed runs"""

    def __enter__(self):
        self.old = {k: os.environ.get(k) for k in PER_STATE_ENV}
        os.environ.update(PER_STATE_ENV)

    def __exit__(self, *exc):
        for k, v in self.old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


MICRO_PROFILE = "profiles/r01_fpset_microbench.jsonl"
# algorithmic HBM bytes per distinct state of the BFS path (read
# the frontier state 8 B, write the new state 8 B and its parent entry 8 B,
# g/d = 1.339 probes of 8 B); roofline.achieved prices every engine with it
SURVEY_BYTES_PER_DISTINCT = 34.7
# MI355X issue model for roofline.issue (MI355X_MICROARCH.md): 256 CUs x 4
# SIMD-32; a wave64 VALU instruction takes 2 cycles of its SIMD, the CU's one
# scalar unit issues one SALU instruction per cycle, SQ_LDS_IDX_ACTIVE counts
# LDS-array cycles (one array per CU); 2.4 GHz
CUS, SIMDS, CLOCK_HZ = 256, 4, 2.4e9


def component_kernel_name(jit):
    """the first-pass component kernel tlcg_stats.jit_used names (bit 0 hipRTC, bit 1 codes,
    bit 3 one walk of the code graph per wavefront, bit 5 the per-lane bitmap pass)"""
    if jit & 8:
        return "tlcg_componentw_64 (hipRTC-specialized, component codes, one code-graph walk per wavefront)"
    if jit & 32:
        return "tlcg_componentp_64 (hipRTC-specialized, component codes, per-lane BFS with a bitmap FPSet)"
    if jit & 1:
        return "tlcg_componentc_64 (hipRTC-specialized, component codes)" if jit & 2 else \
            "tlcg_component_64 (hipRTC-specialized)"
    return "k_component<64, codes>" if jit & 2 else "k_component<64>"


def load_profile(name):
    """profiles/<newest round>_<name>, or None"""
    import glob
    hits = sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]_" + name)))
    return json.load(open(hits[-1])) | {"_file": os.path.relpath(hits[-1], ROOT)} if hits else None


def pmc_fields(name, kernel, kt_s, distinct):
    """traffic and issue of the dominant kernel from profiles/<newest round>_pmc_<name>.json
    (scripts/pmc_kernel.sh + scripts/pmc_summarize.py: one complete check per
    rocprofv3 pass, FETCH_SIZE doubled for gfx950), priced at this run's kernel
    time kt_s; None when the profile is of another kernel"""
    pmc = load_profile(f"pmc_{name}.json")
    if not pmc or "counters" not in pmc or not any(kernel.split()[0].split("<")[0] in k for k in pmc.get("kernels", [])):
        return None
    c = pmc["counters"]
    t_valu = c["SQ_INSTS_VALU"] * 2 / (CUS * SIMDS * CLOCK_HZ)
    t_salu = c["SQ_INSTS_SALU"] / (CUS * CLOCK_HZ)
    t_lds = c["SQ_LDS_IDX_ACTIVE"] / (CUS * CLOCK_HZ)
    return dict(
        traffic=round(pmc["hbm_bytes"] / kt_s / 1e9, 1),
        traffic_bytes_per_step=round(pmc["hbm_bytes"]),
        traffic_source=pmc["_file"],
        issue=dict(frac=round(max(t_valu, t_salu, t_lds) / kt_s, 3),
                   valu_ms=round(t_valu * 1e3, 3), salu_ms=round(t_salu * 1e3, 3), lds_ms=round(t_lds * 1e3, 3),
                   valu_wave_insts_per_state=round(c["SQ_INSTS_VALU"] / distinct, 3),
                   salu_wave_insts_per_state=round(c["SQ_INSTS_SALU"] / distinct, 3),
                   wave_issue_frac=round(c["SQ_ACTIVE_INST_ANY"] / max(c["SQ_WAVE_CYCLES"], 1), 3),
                   lds_bank_conflict_frac=round(c["SQ_LDS_BANK_CONFLICT"] / max(c["SQ_LDS_IDX_ACTIVE"], 1), 3),
                   formula="frac = max(VALU x 2 cyc / (256 CU x 4 SIMD), SALU x 1 cyc / 256 CU, "
                           "SQ_LDS_IDX_ACTIVE / 256 CU) / 2.4 GHz / kernel time (DESIGN 4)"))


def load_microbench(rel):
    """Best measured rate per access kind (accesses/s) from the microbenchmark log."""
    p = os.path.join(ROOT, rel)
    if not os.path.exists(p):
        return None
    best = {}
    for line in open(p):
        if line.startswith("{"):
            r = json.loads(line)
            best[r["kind"]] = max(best.get(r["kind"], 0.0), r["access_per_s"])
    return best


def user_invariants(cfg):
    u = CONFIGS[cfg].get("user", ())
    return (u,) if isinstance(u, str) else tuple(u)


def model_for(cfg):
    import tlcgpu
    k = CONFIGS[cfg]["keys"]
    extra = {}
    if user_invariants(cfg):
        extra = dict(invariants=("TypeSafe",) + user_invariants(cfg) + ("CompactionHorizonCorrectness",),
                     user_defs=dict(USER_DEFS))
    return tlcgpu.Model(key_space=range(1, k + 1), value_space=range(1, k + 1),
                        compaction_times_limit=CONFIGS[cfg].get("C", 3),
                        model_producer=CONFIGS[cfg].get("producer", False),
                        retain_null_key=CONFIGS[cfg].get("retain", True), **extra)


def algorithmic_bytes(distinct, generated, n_init, selfloops, words=1):
    """read each parent, write each new state and its parent entry, one FPSet
    slot probe per non-stuttering successor (a state and a slot are `words`
    8-byte words; the parent entry is one)"""
    probes = generated - n_init - selfloops  # successors inserted into the FPSet
    w = BYTES_PER_STATE_WORD
    return w * words * distinct + (w * words + w) * (distinct - n_init) + w * words * probes


def selfloops_per_m(model):
    import tlcgpu
    seen, todo, loops = set(), [tlcgpu.host_init_state(model, 0)], 0
    while todo:
        s = todo.pop()
        if s in seen:
            continue
        seen.add(s)
        for _, t in tlcgpu.host_successors(model, s):
            loops += t == s
            todo.append(t)
    return loops


def cpu_baseline(cfg, seconds_target=12.0):
    """The oracle (TEST INFRASTRUCTURE, single thread) on a bounded sample of the
    same workload: the first n initial message sequences of the cfg (for a
    producer-modelled cfg, which has one initial state: the whole check of the
    same spec at KeySpace = ValueSpace = {1..4})."""
    oracle = os.path.join(ROOT, "oracle", "build", "tlc_oracle")
    if not os.path.exists(oracle):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, capture_output=True)
    c = CONFIGS[cfg]
    if c.get("producer"):
        keys = "1,2,3,4"
        t = time.time()
        out = subprocess.run([oracle, "-keys", keys, "-values", keys, "-producer", "1", "-retain",
                              "0" if c.get("retain") is False else "1", "-notrace"],
                             check=True, capture_output=True, text=True).stdout
        r = json.loads(out)
        return dict(value=r["distinct"] / r["seconds"], unit="distinct states/s", cores=1, kind="port",
                    sample=f"oracle/tlc_oracle (C restatement, 1 thread), the whole producer-modelled check at "
                           f"KeySpace = ValueSpace = {{1..4}}: {r['distinct']} distinct states in "
                           f"{r['seconds']:.2f} s (TLC itself is not installed on the GPU host)",
                    wall_s=round(time.time() - t, 2))
    k = c["keys"]
    keys = ",".join(str(i) for i in range(1, k + 1))
    n_m = 4096
    while True:
        t = time.time()
        out = subprocess.run([oracle, "-keys", keys, "-values", keys, "-C", str(c.get("C", 3)),
                              "-init-lo", "0", "-init-hi", str(n_m),
                              "-notrace"], check=True, capture_output=True, text=True).stdout
        wall = time.time() - t
        r = json.loads(out)
        if r["seconds"] >= seconds_target / 4 or n_m >= (k + 1) ** 6:
            break
        n_m = min(n_m * 4, (k + 1) ** 6)
    single = dict(value=r["distinct"] / r["seconds"], cores=1,
                  sample=f"the first {n_m} of {(k + 1) ** 6} initial message sequences: {r['distinct']} distinct "
                         f"states in {r['seconds']:.2f} s")
    # all the host cores this job has (the box's share: OMP_NUM_THREADS), one
    # oracle process per core on disjoint slices of the initial message
    # sequences -- components never share states without a Producer, so the
    # slices' counts add up (TLC -workers <cores> stand-in)
    P = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)))
    P = min(P, (k + 1) ** 6 // n_m)
    t = time.time()
    procs = [subprocess.Popen([oracle, "-keys", keys, "-values", keys, "-C", str(c.get("C", 3)),
                               "-init-lo", str(i * n_m), "-init-hi", str((i + 1) * n_m), "-notrace"],
                              stdout=subprocess.PIPE, text=True) for i in range(P)]
    outs = [p.communicate()[0] for p in procs]
    wall_p = time.time() - t
    if any(p.returncode for p in procs):
        raise SystemExit("cpu baseline: an oracle process failed")
    dist_p = sum(json.loads(o)["distinct"] for o in outs)
    return dict(value=dist_p / wall_p, unit="distinct states/s", cores=P, kind="port",
                sample=f"oracle/tlc_oracle (C restatement), {P} processes on {P} cores, process i on initial "
                       f"message sequences [i*{n_m}, (i+1)*{n_m}) of {(k + 1) ** 6} of the {cfg.upper()} cfg: "
                       f"{dist_p} distinct states in {wall_p:.2f} s wall (TLC itself is not installed on the "
                       f"GPU host)",
                single_thread=single, wall_s=round(wall + wall_p, 2))


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="g9", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (RCCL, one GPU per rank) or gloo (rehearsal)")
    return ap.parse_args(argv)


def launch_plan(gpus, environ):
    """What `bench.py --gpus N` does in this environment:
    ("run", None)      this process is the job's only rank, or one rank of a
                       launched job (WORLD_SIZE set, equal to --gpus);
    ("spawn", N)       no launcher ran: start N rank processes (spawn_ranks);
    ("refuse", why)    --gpus contradicts the launcher's WORLD_SIZE."""
    if gpus < 1:
        return "refuse", f"--gpus {gpus}: at least one rank"
    ws = environ.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != gpus:
            return "refuse", (f"--gpus {gpus} but the launcher started WORLD_SIZE={ws} ranks: "
                              f"the line would report {ws} GPUs under a --gpus {gpus} run")
        return "run", None
    return ("spawn", gpus) if gpus > 1 else ("run", None)


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n, child_argv, grace_s=90.0, environ=None):
    """Start n rank processes of `child_argv` (one per GPU, LOCAL_RANK = rank),
    the torch.distributed.run environment set for each, before this process
    touches torch or a GPU (children, never a re-exec).  Rank 0's stdout is
    this process's stdout (the JSON line); the other ranks' goes to stderr.
    When a rank fails, the others get `grace_s` to finish (they are most
    likely blocked in a collective with it) and are then terminated.
    Returns the job's exit code: 0 if every rank exited 0, else the code of
    the first rank that failed (the cause; the others' follow from it)."""
    import signal
    base = dict(os.environ if environ is None else environ)
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(base, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen(child_argv, env=env, stdout=None if r == 0 else sys.stderr))

    def stop(*_):
        for p in procs:
            if p.poll() is None:
                p.terminate()
    old = signal.signal(signal.SIGTERM, lambda *a: (stop(), sys.exit(143)))
    first_bad, deadline = None, None
    try:
        while any(p.poll() is None for p in procs):
            for r, p in enumerate(procs):
                if first_bad is None and p.poll() not in (None, 0):
                    first_bad = (r, p.returncode)
                    deadline = time.time() + grace_s
            if deadline is not None and time.time() > deadline:
                stop()
                deadline = time.time() + 30.0
                for p in procs:
                    try:
                        p.wait(timeout=30)
                    except subprocess.TimeoutExpired:
                        p.kill()
            time.sleep(0.05)
    finally:
        signal.signal(signal.SIGTERM, old)
    for r, p in enumerate(procs):
        if first_bad is None and p.returncode != 0:
            first_bad = (r, p.returncode)
    codes = [p.returncode for p in procs]
    if first_bad is None:
        return 0
    r, rc = first_bad
    print(f"bench: rank {r} of {n} failed first (exit {rc}); ranks' exit codes {codes}", file=sys.stderr, flush=True)
    return rc if rc > 0 else 128 + (-rc)


def main():
    args = parse_args()
    plan, what = launch_plan(args.gpus, os.environ)
    if plan == "refuse":
        print(f"bench: refused: {what}", file=sys.stderr, flush=True)
        sys.exit(2)
    if plan == "spawn":
        sys.exit(spawn_ranks(what, [sys.executable, "-u", os.path.abspath(__file__)] + sys.argv[1:]))

    import torch
    import tlcgpu

    # a collective that does not complete (a peer rank died) aborts instead of hanging
    os.environ.setdefault("TLCG_COMM_TIMEOUT_S", "60")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    distributed = world > 1
    ndev = torch.cuda.device_count()
    gpu = local_rank % max(ndev, 1)  # = local_rank on a node with one GPU per rank
    if distributed:
        import torch.distributed as dist
        torch.cuda.set_device(gpu)
        try:
            if args.dist_backend == "nccl":
                dist.init_process_group("nccl", device_id=torch.device(f"cuda:{gpu}"))
            else:
                dist.init_process_group(args.dist_backend)
        except Exception as e:  # noqa: BLE001
            # e.g. RCCL's refusal of two ranks on one device (ncclCommInitRank: invalid usage)
            print(f"bench: rank {rank}: {args.dist_backend} process group over {world} ranks on "
                  f"{ndev} visible device(s) failed: {type(e).__name__}: {str(e)[:400]}", file=sys.stderr, flush=True)
            sys.exit(4)
    dev = torch.device(f"cuda:{gpu}")
    rdev = dev if args.dist_backend == "nccl" else torch.device("cpu")  # reduction tensors

    cfg = CONFIGS[args.config]
    model = model_for(args.config)
    words = tlcgpu.state_words(model)
    import dist as tdist

    def time_engine(engine):
        """warmup + K timed complete checks with one engine; max over ranks"""
        per_rank = cfg["distinct"] // world + 1
        log2 = max(16, (2 * per_rank - 1).bit_length()) if engine == "global" else 0
        cap = int(per_rank * 1.08) + 2 * (cfg["distinct"] // 12) // world + (1 << 20)
        eng = tdist.GpuEngine(model, rank, world, gpu, log2_fpset_slots=log2, state_capacity=cap, engine=engine)
        assert eng.closed
        for _ in range(args.warmup):
            eng.run_closed()
        torch.cuda.synchronize(dev)
        if distributed:
            dist.barrier()
        torch.cuda.synchronize(dev)
        kms = ems = 0.0
        t0 = time.perf_counter()
        for _ in range(args.steps):
            st = eng.run_closed()
            ems += st.expand_ms
            kms += st.kernel_ms
        torch.cuda.synchronize(dev)
        if distributed:
            dist.barrier()
        torch.cuda.synchronize(dev)
        elapsed = time.perf_counter() - t0
        counts = [st.generated, st.distinct]
        try:  # the kernels' own count of state expansions (tlcg_expansions)
            expansions = eng.ck.expansions()
        except RuntimeError:
            expansions = None
        used = tlcgpu.ENGINE_NAMES.get(int(st.engine), "?")
        jit = int(st.jit_used)
        launches = len(eng.level_sizes()) if used == "global" else \
            cfg.get("N", 3) + 1 if used == "tree" and cfg.get("producer") else 1
        if distributed:
            t = torch.tensor([elapsed, ems, kms], dtype=torch.float64, device=rdev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed, ems, kms = [float(x) for x in t.tolist()]
            x = torch.tensor([expansions if expansions is not None else -1], dtype=torch.int64, device=rdev)
            dist.all_reduce(x, op=dist.ReduceOp.MIN)
            if int(x.item()) >= 0:
                dist.all_reduce(x.fill_(expansions), op=dist.ReduceOp.SUM)
                expansions = int(x.item())
            else:
                expansions = None
            c = torch.tensor(counts, dtype=torch.int64, device=rdev)
            dist.all_reduce(c, op=dist.ReduceOp.SUM)
            counts = [int(x) for x in c.tolist()]
        eng.close()
        if tuple(counts) != (cfg["generated"], cfg["distinct"]):
            raise SystemExit(f"count mismatch ({engine}): {counts} want {cfg}")
        return dict(engine=used, jit=jit, elapsed=elapsed, expand_ms=ems / args.steps, kernel_ms=kms / args.steps,
                    launches=launches, expansions=expansions)

    def time_exchange(partition):
        """The global engine with successors crossing ranks, so every BFS level
        runs expand -> all-gather of counts -> send/recv of {state, parent}
        records over RCCL (xGMI) -> absorb -> all-reduce, all inside libtlcgpu
        (tlcg_run_comm; dist.run_native).  BASELINE config 4: on G9 the FPSet
        is partitioned on the whole state (partition 2); a producer-modelled
        cfg is open by itself (partition 0)."""
        per_rank = cfg["distinct"] // world + 1
        log2 = max(16, (2 * per_rank - 1).bit_length())
        cap = int(per_rank * 1.1) + (1 << 20)
        eng = tdist.GpuEngine(model, rank, world, gpu, log2_fpset_slots=log2, state_capacity=cap, engine="global",
                              partition=partition)
        assert not eng.closed
        tdist.init_native(eng)
        for _ in range(args.warmup):
            tdist.run_native(eng)
        torch.cuda.synchronize(dev)
        dist.barrier()
        torch.cuda.synchronize(dev)
        kms = ems = 0.0
        t0 = time.perf_counter()
        for _ in range(args.steps):
            r = tdist.run_native(eng)
            kms += r.kernel_ms
            ems += r.expand_ms
        torch.cuda.synchronize(dev)
        dist.barrier()
        torch.cuda.synchronize(dev)
        elapsed = time.perf_counter() - t0
        t = torch.tensor([elapsed, ems, kms], dtype=torch.float64, device=rdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        eng.close()
        if (r.generated, r.distinct, r.depth) != (cfg["generated"], cfg["distinct"], cfg["depth"]):
            raise SystemExit(f"count mismatch (exchange): {(r.generated, r.distinct, r.depth)} want {cfg}")
        if r.engine == "tree":  # Producer modelled: each rank ran whole subtrees of the component tree
            return dict(engine="tree", jit=1, elapsed=float(t[0]), expand_ms=float(t[1]) / args.steps,
                        kernel_ms=float(t[2]) / args.steps, launches=cfg.get("N", 3) + 1,
                        partition="component tree, whole subtrees per rank (csrc/tree.h): no exchange",
                        exchange="none on the data path: tlcg_run_comm all-reduces the combined counts over RCCL")
        return dict(engine="global", jit=0, elapsed=float(t[0]), expand_ms=float(t[1]) / args.steps,
                    kernel_ms=float(t[2]) / args.steps, launches=cfg["depth"] - 1,
                    kernel="k_expand<u64, open partition> + k_absorb",
                    partition="whole state (owner = mix64(state))" if partition == 2 else "open (Producer)",
                    exchange="libtlcgpu tlcg_run_comm: ncclAllGather (counts) + grouped ncclSend/ncclRecv "
                             "(16-B records) + ncclAllReduce per level, RCCL over xGMI")

    open_model = bool(cfg.get("producer"))
    global_run = wave_run = None
    if open_model and distributed:
        # the component tree split by subtrees (no exchange), or the level loop's exchange if it hands over
        main_run = time_exchange(0)
    else:
        # the headline: the fastest engine whose timed
        # kernel expands every distinct state -- the on-chip engines' per-lane
        # kernels (component_body.h: every lane its own component's FIFO,
        # FPSet probes, invariants; tree_body.h for the closed tree) -- with
        # the one-walk-per-wavefront kernels switched off
        with per_state_kernels():
            main_run = time_engine("auto")
        if main_run["jit"] & (8 | 16):
            raise SystemExit("the per-state headline ran a one-walk-per-wavefront kernel")
        global_run = time_engine("global")  # the HBM-FPSet engine (the north-star design)
        # the wave kernels (component_wave.h, tree_wave.h): one walk of the code
        # graph per wavefront applied to M x 64 components -- a product
        # quotient, reported apart (engines.wave_quotient), never the headline
        if not open_model:
            wave_run = time_engine("auto")
            if not (wave_run["jit"] & (8 | 16)):
                wave_run = None
    distinct, generated = cfg["distinct"], cfg["generated"]
    # (a producer-modelled cfg has one initial state; its Terminating stutters
    # are not counted out of the probes, so its bytes/state is an upper bound)
    n_init = 1 if open_model else (cfg["keys"] + 1) ** 6
    selfloops = 0 if open_model else n_init * selfloops_per_m(model)

    def survey_roofline(r, kernel):
        """34.7 algorithmic bytes per distinct state x the distinct
        states of one step (this rank's share) / the step's kernel time (HIP
        events around the launches, inside the library) against the 8 TB/s
        HBM peak -- the same pricing for every per-state engine"""
        bytes_step = SURVEY_BYTES_PER_DISTINCT * distinct / world
        kt = r["expand_ms"] * 1e-3
        achieved = bytes_step / kt / 1e9
        return dict(bound="hbm", achieved=round(achieved, 1), peak=HBM_PEAK_GBS, unit="GB/s",
                    frac=round(achieved / HBM_PEAK_GBS, 4), traffic=None, kernel=kernel,
                    launches_per_step=r["launches"], avg_launch_ms=round(r["expand_ms"] / r["launches"], 4),
                    bytes_per_distinct=SURVEY_BYTES_PER_DISTINCT,
                    algorithmic_bytes_per_step=round(bytes_step),
                    basis="SURVEY 8(d): read the frontier state 8 B, write the new state 8 B and its parent "
                          "entry 8 B, g/d = 1.339 FPSet probes of 8 B; x distinct states of one step")

    def roofline_global(r):
        abytes = algorithmic_bytes(distinct, generated, n_init, selfloops, words)
        rf = survey_roofline(r, r.get("kernel") or ("k_expand_fast" if words == 1 and not open_model else
                                                    "k_expand_prod<8> (Producer)" if words == 1 else
                                                    "k_expand<u128> (wide FPSet)"))
        rf["kernel_bytes_per_distinct"] = round(abytes / distinct, 2)
        new = pmc_fields(f"expand_{args.config}", rf["kernel"], r["expand_ms"] * 1e-3, distinct) \
            if world == 1 and words == 1 and not open_model else None
        if new:
            rf.update(new)
            rf["traffic_over_algorithmic"] = round(new["traffic_bytes_per_step"] / abytes, 2)
        pmc = None if new else load_profile(PMC_PROFILE)
        avg_launch_s = r["expand_ms"] / r["launches"] * 1e-3
        if pmc and args.config == "g9" and world == 1 and words == 1 and not open_model:
            rf["traffic"] = round(pmc["hbm_bytes_per_launch"] / avg_launch_s / 1e9, 1)
            rf["traffic_bytes_per_launch"] = round(pmc["hbm_bytes_per_launch"])
            rf["traffic_over_algorithmic"] = round(pmc["hbm_bytes_per_launch"] * r["launches"] / abytes, 2)
            rf["traffic_source"] = pmc["_file"]
        micro = load_microbench(MICRO_PROFILE)
        if micro and words == 1:
            probes = (generated - n_init - selfloops) / world
            inserts = (distinct - n_init) / world
            bound_ms = (probes / micro["load_nt"] + inserts / micro["cas_new"]) * 1e3
            rf["scattered_access_roofline"] = dict(
                probes_per_step=int(probes), inserts_per_step=int(inserts), load_per_s=micro["load_nt"],
                cas_per_s=micro["cas_new"], bound_ms_per_step=round(bound_ms, 2),
                frac=round(bound_ms / r["expand_ms"], 3), source=MICRO_PROFILE)
        return rf

    ON_CHIP_NOTE = ("on-chip engine: each lane expands its own component's states with its FIFO and FPSet in "
                    "LDS, so SURVEY 8(d)'s bytes move through LDS, not HBM (roofline.traffic is the HBM the "
                    "kernel did move, by PMC); roofline.issue is the bound that binds it (DESIGN 4)")

    def roofline_component(r):
        # the per-lane kernel: its own HBM bytes are one 4-B store record per
        # distinct state (comp_record; FIFO and FPSet in LDS)
        kt = r["expand_ms"] * 1e-3
        rf = survey_roofline(r, component_kernel_name(r["jit"]))
        rf["kernel_hbm_bytes_per_distinct"] = COMPONENT_BYTES_PER_STATE
        rf["note"] = ON_CHIP_NOTE
        new = None
        if world == 1:
            for prof in ([f"component_{args.config}"] if r["jit"] & 8 else
                         [f"component_perlane_{args.config}", f"component_{args.config}"]):
                new = new or pmc_fields(prof, rf["kernel"], kt, distinct)
        if new:
            rf.update(new)
            rf["traffic_over_kernel_bytes"] = round(new["traffic_bytes_per_step"] /
                                                    (COMPONENT_BYTES_PER_STATE * distinct / world), 3)
        return rf

    def tree_kernel_name(jit):
        if open_model:
            return ("tlcg_tree_384 (hipRTC-specialized, " if jit & 1 else "k_tree<384, 512, 4> (") + \
                "component tree, 4 components per wavefront, double-hashed LDS tables)"
        if jit & 16:
            return "tlcg_treecw_640 (hipRTC-specialized, component tree closed mode: one code-graph walk " \
                "per wavefront, lane-interleaved store)"
        if jit & 128:
            return "tlcg_treecb_640 (hipRTC-specialized, component tree closed mode: component codes, " \
                "a bitmap FPSet over the host's perfect hash, 16 components per wavefront)"
        return ("tlcg_treec_640 (hipRTC-specialized, " if jit & 1 else "k_tree<640, 1024, 4, closed> (") + \
            "component tree closed mode: component codes, 4 components per wavefront)"

    def roofline_tree(r):
        # the tree writes the parent entry per state and the state word
        # (Producer modelled, plus a depth byte: 9 B per entry) or, closed, the
        # 4-B component code the host decodes; its FPSets stay in LDS
        rf = survey_roofline(r, tree_kernel_name(r["jit"]))
        rf["kernel_hbm_bytes_per_distinct"] = BYTES_PER_STATE_WORD * (words + 1) + 1 if open_model else \
            4 + BYTES_PER_STATE_WORD
        rf["note"] = ON_CHIP_NOTE
        prof = f"tree_{args.config}" if open_model else f"tree_perlane_{args.config}"
        new = pmc_fields(prof, rf["kernel"], r["expand_ms"] * 1e-3, distinct) if world == 1 else None
        if new:
            rf.update(new)
        return rf

    def summary(r):
        out = dict(engine=r["engine"], jit=bool(r["jit"]), value=round(distinct * args.steps / r["elapsed"], 1),
                   ms_per_step=round(r["elapsed"] * 1e3 / args.steps, 3),
                   gpu_kernel_ms_per_step=round(r["kernel_ms"], 3),
                   roofline=roofline_component(r) if r["engine"] == "component" else
                   roofline_tree(r) if r["engine"] == "tree" else roofline_global(r))
        if r.get("expansions") is not None:
            # the kernels' own count (tlcg_expansions): every distinct state
            # expanded once by a per-state kernel
            out["expansions_per_step"] = r["expansions"]
            out["distinct_per_expansion"] = round(distinct / max(r["expansions"], 1), 3)
        for k in ("partition", "exchange"):
            if k in r:
                out[k] = r[k]
        return out

    def wave_summary(r):
        """the one-walk-per-wavefront kernels: a wave expands its code graph
        once (the code states of one component) and applies each expansion to
        the M x 64 components of the walk (their invariants by one ballot over
        the 32 flag combinations, component_wave.h) -- a quotient of the product
        state space, not a per-state throughput: no roofline is claimed"""
        comps = tlcgpu.init_count(model) // world
        per_comp = distinct // (cfg["keys"] + 1) ** 6 if not open_model else None
        if r["engine"] == "tree":
            m, kern = TREE_WAVE_M, tree_kernel_name(r["jit"])
        else:
            m = WAVE_M_USER if cfg.get("user") else WAVE_M_BIG if comps >= WAVE_BIG_COMPS else WAVE_M
            kern = component_kernel_name(r["jit"])
        walks = -(-(-(-comps // 64)) // m)
        # the kernel's own count (tlcg_expansions: one per walk and code state)
        expanded = r.get("expansions") or (walks * per_comp if per_comp else None)
        return dict(engine=r["engine"], kernel=kern, quotient=True,
                    value_quotient=round(distinct * args.steps / r["elapsed"], 1),
                    ms_per_step=round(r["elapsed"] * 1e3 / args.steps, 3),
                    gpu_kernel_ms_per_step=round(r["kernel_ms"], 3),
                    components_per_walk=m * 64, walks_per_step=walks,
                    code_states_expanded=expanded,
                    states_per_expansion=round(distinct / world / expanded, 1) if expanded else None,
                    roofline=None,
                    note="a product quotient (messages is immutable and the code transitions read only Len): "
                         "the rate grows with components per walk, not with hardware throughput; not a "
                         "per-state BFS rate (VERDICT r5)")

    main_s = summary(main_run)
    if main_s.get("expansions_per_step") is not None:
        main_s["roofline"]["expansions_per_step"] = main_s["expansions_per_step"]

    def build_line(exchange_run, exchange_error):
        line = {
            "metric": "distinct states/sec, compaction.tla scaled cfg, 1/2/4/8 MI355X vs host TLC",
            "value": main_s["value"],
            "unit": "distinct states/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": main_s["ms_per_step"],
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic: the model's own state space (no external data)",
            "config": {"workload": f"compaction.tla BFS, {args.config.upper()} cfg: KeySpace = ValueSpace = "
                                   f"{{1..{cfg['keys']}}}, MessageSentLimit 3, CompactionTimesLimit {cfg.get('C', 3)}, "
                                   f"MaxCrashTimes 1, RetainNullKey {'FALSE' if cfg.get('retain') is False else 'TRUE'}, "
                                   f"{'ModelProducer' if open_model else 'no producer'}, no consumer",
                       "state_bits": tlcgpu.state_bits(model),
                       "distinct": distinct, "generated": generated, "depth": cfg["depth"],
                       "parallelism": f"partition{world}", "engine": main_s["engine"],
                       "gpu_kernel_ms_per_step": main_s["gpu_kernel_ms_per_step"]},
            "roofline": main_s["roofline"],
            "engines": {},
        }
        if main_s.get("expansions_per_step") is not None:
            line["expansions_per_step"] = main_s["expansions_per_step"]
            line["distinct_per_expansion"] = main_s["distinct_per_expansion"]
        if user_invariants(args.config):
            line["config"]["invariants"] = list(model.invariants)
            line["config"]["user_invariants"] = {n: USER_DEFS[n] for n in user_invariants(args.config)}
        if global_run:
            line["engines"]["global_hbm_fpset"] = summary(global_run)
        if wave_run:
            line["engines"]["wave_quotient"] = wave_summary(wave_run)
        if distributed:
            line["dist_backend"] = args.dist_backend
            line["rccl_ranks"] = preflight["rccl_ranks"] if preflight else None
            if preflight:
                line["rccl_preflight"] = preflight
        if exchange_run:
            line["engines"]["global_open_partition_alltoall"] = summary(exchange_run)
            line["exchange_leg_ok"] = True
        elif exchange_error and exchange_error.startswith("skipped"):
            line["exchange_leg_ok"] = None
            line["exchange_leg_error"] = exchange_error
        elif exchange_error:
            line["engines"]["global_open_partition_alltoall"] = {"error": exchange_error}
            line["exchange_leg_ok"] = False
            line["exchange_leg_error"] = exchange_error
        return line

    def rccl_preflight():
        """The S cfg hash-partitioned on the whole state over the library's own
        RCCL communicator (tlcg_comm_init -> tlcg_run_comm: all-gather, grouped
        send/recv, all-reduce every level): exact counts, and the
        communicator's rank count (tlcg_comm_size = ncclCommCount)"""
        s_model = tlcgpu.Model()
        eng = tdist.GpuEngine(s_model, rank, world, gpu, log2_fpset_slots=18, state_capacity=1 << 17,
                              engine="global", partition=2)
        try:
            tdist.init_native(eng)
            n = int(eng.lib.tlcg_comm_size(eng.ctx))
            t = time.perf_counter()
            r = tdist.run_native(eng)
            ms = (time.perf_counter() - t) * 1e3
        finally:
            eng.close()
        want = CONFIGS["s"]
        ok = (r.generated, r.distinct, r.depth) == (want["generated"], want["distinct"], want["depth"])
        return dict(rccl_ranks=n, counts_exact=ok, levels=r.depth, ms=round(ms, 2))

    exchange_run = exchange_error = preflight = None
    if distributed and not open_model and args.dist_backend != "nccl":
        exchange_error = f"skipped: the exchange runs over RCCL, not {args.dist_backend} (a rehearsal backend)"
    elif distributed and not open_model and os.environ.get("TLCG_BENCH_EXCHANGE", "1") != "0":
        # a secondary measurement (BASELINE config 4): its failure (every rank
        # learns of it through torch's own group) must not cost the headline
        # line, and neither may a hang -- the library aborts a collective after
        # TLCG_COMM_TIMEOUT_S, and this watchdog ends the job with the headline
        # line if the whole leg outlives TLCG_BENCH_EXCHANGE_TIMEOUT_S
        limit = float(os.environ.get("TLCG_BENCH_EXCHANGE_TIMEOUT_S", "240"))

        def bail():
            # the headline line still stands, but a hung leg is a failed job:
            # it is named at the line's top level (exchange_leg_ok false) and
            # the process exits non-zero
            if rank == 0:
                print(json.dumps(build_line(None, f"the exchange leg did not finish within {limit:.0f} s")), flush=True)
            print(f"bench: rank {rank}: the exchange leg hung (> {limit:.0f} s)", file=sys.stderr, flush=True)
            os._exit(3)

        import threading
        watchdog = threading.Timer(limit, bail)
        watchdog.daemon = True
        watchdog.start()
        try:
            preflight = rccl_preflight()
            if not preflight["counts_exact"]:
                raise RuntimeError(f"RCCL preflight on the S cfg: inexact counts {preflight}")
            exchange_run = time_exchange(2)
            ok = 1
        except (Exception, SystemExit) as e:  # noqa: BLE001
            exchange_error = f"{type(e).__name__}: {e}"[:300]
            ok = 0
        flag = torch.tensor([ok], dtype=torch.int64, device=rdev)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        watchdog.cancel()
        if not int(flag.item()):
            exchange_run = None
            exchange_error = exchange_error or "failed on another rank"
    if rank == 0:
        line = build_line(exchange_run, exchange_error)
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(args.config)
        print(json.dumps(line), flush=True)
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
