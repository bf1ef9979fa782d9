/*
 * include/tlcgpu.h -- C ABI of libtlcgpu.so, the MI355X (gfx950) BFS safety
 * checker for the Pulsar topic-compaction spec (/root/reference/compaction.tla).
 *
 * This is the drop-in boundary: the entry points are the calls TLC's model
 * checker core makes on the path the HIP kernels replace.  TLC (tla2tools.jar)
 * is not part of the reference repo (its .gitignore:3 ignores *.jar), so the
 * TLC classes are cited by name; the spec lines are cited as file:line.
 *
 *   tlcg_check_model  <- ModelChecker.checkAssumptions: the ASSUME of
 *                        compaction.tla:25-35 on the bound constants
 *   tlcg_create       <- new ModelChecker(...) + FPSet / StateQueue / TLCTrace
 *                        allocation (tlc2.tool.ModelChecker, tlc2.tool.fp.FPSet)
 *   tlcg_init         <- ModelChecker.doInit: Init, compaction.tla:188-202,
 *                        FPSet.put + invariant check of each initial state
 *   tlcg_step_level   <- one BFS level of tlc2.tool.Worker.run: Next
 *                        (compaction.tla:216-231), fingerprint, FPSet.put,
 *                        invariants (compaction.cfg:25-31), enqueue, deadlock
 *   tlcg_run          <- ModelChecker.runTLC (levels until done or error)
 *   tlcg_trace        <- TLCTrace.getTrace (parent-pointer walk)
 *   tlcg_decode       <- TLCStateMut.toString (TLC value syntax)
 *   tlcg_expand / tlcg_outbox / tlcg_inbox / tlcg_absorb / tlcg_end_level
 *                     <- the per-level exchange of a fingerprint-partitioned
 *                        FPSet (TLC's distributed tlc2.tool.fp.FPSetManager),
 *                        one rank per GPU
 *
 * Conventions: plain C, no exceptions cross the ABI, buffers are owned by the
 * caller, one host thread per context.  A negative return is an error whose
 * text tlcg_last_error() returns.  Device pointers handed out by
 * tlcg_outbox/tlcg_inbox are valid until the next call on the context.
 */
#ifndef TLCGPU_H
#define TLCGPU_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TLCG_ABI_VERSION 4
#define TLCG_MAX_SET 63 /* largest KeySpace / ValueSpace */
#define TLCG_MAX_INV 8

/* invariants the spec defines (compaction.tla:236,253,259,280) */
enum {
  TLCG_INV_TYPESAFE = 0,            /* TypeSafe */
  TLCG_INV_COMPACTED_LEDGER_LEAK = 1, /* CompactedLedgerLeak */
  TLCG_INV_HORIZON_CORRECTNESS = 2, /* CompactionHorizonCorrectness */
  TLCG_INV_DUP_NULLKEY_MESSAGE = 3, /* DuplicateNullKeyMessage */
  /* TLCG_INV_USER + j: the j-th definition of tlcg_model.user_defs (an
   * invariant the user added to the module: BASELINE config 5) */
  TLCG_INV_USER = 16
};

/* Next disjuncts, source order (compaction.tla:216-231); -1 = Init */
enum {
  TLCG_ACT_INIT = -1,
  TLCG_ACT_PRODUCER = 0,
  TLCG_ACT_PHASE_ONE,
  TLCG_ACT_PHASE_TWO_WRITE,
  TLCG_ACT_PHASE_TWO_UPDATE_CONTEXT,
  TLCG_ACT_PHASE_TWO_UPDATE_HORIZON,
  TLCG_ACT_PHASE_TWO_PERSIST_CURSOR,
  TLCG_ACT_PHASE_TWO_DELETE_LEDGER,
  TLCG_ACT_BROKER_CRASH,
  TLCG_ACT_CONSUMER,
  TLCG_ACT_TERMINATING
};

/* run status */
enum {
  TLCG_RUNNING = 0,
  TLCG_DONE = 1,             /* "Model checking completed. No error has been found." */
  TLCG_VIOLATION = 2,        /* "Invariant X is violated." */
  TLCG_DEADLOCK = 3,         /* "Deadlock reached." */
  TLCG_ACTION_ERROR = 4,     /* evaluation error while computing a successor */
  TLCG_INVARIANT_ERROR = 5   /* evaluation error while evaluating an invariant */
};

/* The constants of compaction.tla:10-18 as bound by a TLC cfg
 * (compaction.cfg:2-11), plus the INVARIANTS list (compaction.cfg:25-31). */
typedef struct tlcg_model {
  int32_t msg_sent_limit;          /* MessageSentLimit */
  int32_t compaction_times_limit;  /* CompactionTimesLimit */
  int32_t consume_times_limit;     /* ConsumeTimesLimit */
  int32_t max_crash_times;         /* MaxCrashTimes */
  uint8_t model_consumer;          /* ModelConsumer */
  uint8_t model_producer;          /* ModelProducer */
  uint8_t retain_null_key;         /* RetainNullKey */
  uint8_t check_deadlock;          /* 1 unless TLC's -deadlock flag */
  int32_t n_keys, n_values;        /* |KeySpace|, |ValueSpace| */
  int64_t keys[TLCG_MAX_SET];      /* KeySpace elements (any order; 0 is reserved) */
  int64_t values[TLCG_MAX_SET];    /* ValueSpace elements */
  int32_t n_invariants;
  int32_t invariants[TLCG_MAX_INV]; /* TLCG_INV_* in cfg order */
  /* Definitions user invariants may use (NULL: none), as TLA+ text: each
   * definition is a header line "@@DEF <name> [<param> ...] [@<line>]"
   * followed by its body as written in the module (columns kept: bulleted
   * /\ and \/ lists are read by column).  TLCG_INV_USER + j names the j-th
   * definition.  A user invariant is a state predicate over the spec's
   * variables and constants (the subset user_inv.cpp documents); one outside
   * it is refused at tlcg_create / tlcg_check_model, never checked
   * approximately.  Every engine and any number of ranks check them: the
   * on-chip engines (component, component tree) as device code generated
   * from the compiled program into their run-time specialized kernels, the
   * global engine in a check kernel over each new level (TLCG_JIT=0 leaves
   * such models to the global engine).  The text is copied by tlcg_create.  (ModelChecker's
   * invariant list, compaction.cfg:25-31, with invariants the user defined
   * in the .tla, compaction.tla:236-294 being the spec's own.) */
  const char* user_defs;
} tlcg_model;

typedef struct tlcg_opts {
  int32_t device;            /* HIP device ordinal */
  int32_t log2_fpset_slots;  /* FPSet size (8-byte slots); 0 = auto, grows on demand */
  uint64_t state_capacity;   /* states kept for traces; 0 = auto, grows on demand */
  int32_t tlc_order;         /* 1: order every level like TLC -workers 1 (exact TLC trace) */
  int32_t rank, world;       /* fingerprint partition: this context owns rank of world */
  int32_t partition;         /* 0 auto (by `messages` when it is immutable), 1 by `messages`, 2 whole state */
  int32_t engine;            /* TLCG_ENGINE_*: 0 auto, 1 global HBM FPSet, 2 component (closed partitions),
                                3 component tree (Producer modelled) */
  /* Global engine: move committed levels other than the frontier (states and
   * parent log, the trace) to pinned host memory instead of growing the
   * device state store past device_store_cap states (0: past what free HBM
   * allows).  TLC spills its trace and queue to disk the same way
   * (StateQueue, TLCTrace); counts, levels and traces are unchanged. */
  int32_t spill;
  uint64_t device_store_cap;
  /* Host FPSet tier (TLC's DiskFPSet), global engine, <= 63-bit states: when
   * the HBM FPSet would grow past 2^log2_fpset_max slots (0: past what free
   * HBM allows), the states it holds move to a sorted run in host memory,
   * summarized in HBM by a blocked Bloom filter, and the HBM table restarts
   * empty.  Each level's new states are checked against the host runs where
   * the filter says "maybe".  Counts, levels and traces are unchanged. */
  int32_t fpset_spill;
  int32_t log2_fpset_max;
  /* 1: keep TLC's outdegree histogram (tlcg_outdegree).  It costs the
   * component kernel about 9 % on G9, so it is off unless asked for. */
  int32_t outdegree;
  int32_t reserved[1];
} tlcg_opts;

/* BFS engines.  GLOBAL: level-synchronous BFS over one HBM FPSet (64-bit CAS),
 * any model.  COMPONENT: when `messages` is immutable (no Producer) every
 * initial message sequence spans an independent component; a wavefront lane
 * runs TLC's FIFO BFS on one component with an on-chip FPSet.  Same counts,
 * same TLC-order trace; used by AUTO when every component fits on chip. */
enum { TLCG_ENGINE_AUTO = 0, TLCG_ENGINE_GLOBAL = 1, TLCG_ENGINE_COMPONENT = 2,
       TLCG_ENGINE_TREE = 3 /* the component tree of a Producer-modelled spec (auto picks it; falls back to
                               the global engine on an error to report or a component past 1024 states) */ };

typedef struct tlcg_stats {
  uint64_t generated;        /* "states generated" (initial states included) */
  uint64_t distinct;         /* "distinct states found" (this rank) */
  uint64_t frontier;         /* states of the newest level ("left on queue" when stopped) */
  int32_t depth;             /* BFS levels so far, the initial level counting as 1 */
  int32_t status;            /* TLCG_* status */
  int32_t invariant;         /* index into tlcg_model.invariants of the failing one, else -1 */
  int32_t action;            /* TLCG_ACT_* of the failing step (or -1) */
  uint64_t event_gidx;       /* state index of the violating/deadlocked state, or of the
                                parent of a failing action */
  double fp_collision_optimistic; /* TLC's estimate d*(g-d)/2^64 (the set itself is exact) */
  double kernel_ms;          /* total device time of the BFS kernels so far (HIP events) */
  double expand_ms;          /* device time of the expand kernels alone */
  uint64_t levels_redone;    /* levels re-run after an FPSet / store growth */
  uint64_t engine;           /* TLCG_ENGINE_* that produced these numbers */
  uint64_t jit_used;         /* bit 0: the layout-specialized (hipRTC) component kernels ran;
                                bit 1: the component engine ran component codes (16-bit lanes);
                                bit 2: user invariants: the global engine's check is device code
                                (hipRTC, tlcg_user_check), not the interpreter;
                                bit 3: the code pass walked each code graph once per wavefront
                                for its components (tlcg_componentw_64, component_wave.h);
                                bit 4: the component tree's closed mode did the same
                                (tlcg_treecw_640, tree_wave.h: its store is lane-interleaved);
                                bit 5: the code pass ran per lane with a bitmap FPSet over a slot
                                hash injective on the component code set (tlcg_componentp_64,
                                component_lane.h);
                                bit 6: the global engine's fast level ran layout-specialized
                                (tlcg_expand_fast_2, expand_fast.h);
                                bit 7: the component tree's closed pass ran with a bitmap FPSet
                                over the host's perfect hash (tlcg_treecb_640, tree_body.h) */
  uint64_t host_states;      /* committed states spilled to host memory (tlcg_opts.spill) */
  uint64_t fpset_host_states; /* states held by the host FPSet tier (tlcg_opts.fpset_spill) */
  uint64_t transport;        /* multi-rank runs: 1 host threads + device copies, 2 RCCL; 0 one context */
  uint64_t tlc_exact;        /* 1: the run stopped on an error and its trace (tlcg_trace_words) and
                                tlcg_tlc_stop_stats are TLC -workers 1's: a TLC-order run (also the
                                one a component-tree error switches to on one rank), or an on-chip
                                engine's error on a closed partition (one rank) */
} tlcg_stats;

typedef struct tlcg_ctx tlcg_ctx;

int tlcg_abi_version(void);
/* ASSUME (compaction.tla:25-35) + packing check.  0 ok, <0 with a message in err. */
int tlcg_check_model(const tlcg_model* m, char* err, int32_t cap);
/* bits of the packed state for these constants (<= 126 supported) */
int tlcg_state_bits(const tlcg_model* m);
/* uint64 words per packed state: 1 (<= 63 bits) or 2 (a wide layout, <= 126
 * bits).  Every entry point that passes a state as one uint64_t refuses wide
 * layouts; its *_words twin takes `words` uint64s per state, low word first. */
int tlcg_state_words(const tlcg_model* m);
/* number of initial states (Init, compaction.tla:188-202) */
uint64_t tlcg_init_count(const tlcg_model* m);

int tlcg_create(const tlcg_model* m, const tlcg_opts* o, tlcg_ctx** out);
void tlcg_destroy(tlcg_ctx* c);
const char* tlcg_last_error(const tlcg_ctx* c);

/* (Re)starts a run: clears the FPSet and the queue, then Init. */
int tlcg_init(tlcg_ctx* c, tlcg_stats* st);
/* One BFS level (world == 1): expand, dedup, check, enqueue. */
int tlcg_step_level(tlcg_ctx* c, tlcg_stats* st);
/* tlcg_init + tlcg_step_level until status != TLCG_RUNNING (world == 1). */
int tlcg_run(tlcg_ctx* c, tlcg_stats* st);

/* Per-level distinct counts of this rank, level 0 = initial states. */
int tlcg_level_sizes(tlcg_ctx* c, uint64_t* out, int32_t cap, int32_t* n);
/* Trace to the event state: states[0] is initial; actions[i] is the step that
 * produced states[i] (TLCG_ACT_INIT for i = 0).  world == 1 only. */
int tlcg_trace(tlcg_ctx* c, uint64_t* states, int32_t* actions, int32_t cap, int32_t* len);
/* One stored state and its parent reference ((rank << 56) | parent_gidx << ord_bits | ordinal,
 * or ~0 for an initial state). */
int tlcg_state_at(tlcg_ctx* c, uint64_t gidx, uint64_t* state, uint64_t* parent_ref);
/* Copy stored states [first, first + n) to host memory. */
int tlcg_copy_states(tlcg_ctx* c, uint64_t first, uint64_t n, uint64_t* out);
/* the same for either width (states hold tlcg_state_words() uint64s each) */
int tlcg_trace_words(tlcg_ctx* c, uint64_t* states, int32_t* actions, int32_t cap, int32_t* len);
int tlcg_state_at_words(tlcg_ctx* c, uint64_t gidx, uint64_t* state, uint64_t* parent_ref);
int tlcg_copy_states_words(tlcg_ctx* c, uint64_t first, uint64_t n, uint64_t* out);
/* TLC's "G states generated, D distinct states found, Q states left on
 * queue." at the moment a one-worker TLC run stops on the error this context
 * found (TLC prints it after the trace; replaces the end-of-level counts
 * tlcg_stats carries at an error).  Follows ModelChecker.doNext: FIFO
 * dequeue, Next disjuncts in order, each action's StateVec counted before its
 * successors are inserted and checked, stop at the first violating new state,
 * at a failing action (its successors uncounted) or after a deadlocked
 * state's actions.  Needs a global-engine run in TLC order (tlcg_opts.tlc_order,
 * world 1); refused after tlcg_recover.  [TLC-ext: restated from TLC's
 * worker loop, not confirmable without TLC.] */
int tlcg_tlc_stop_stats(tlcg_ctx* c, uint64_t* generated, uint64_t* distinct, uint64_t* left_on_queue);
/* TLC's outdegree statistics of a completed check ("The average outdegree of
 * the complete state graph is M (minimum is A, the maximum B and the 95th
 * percentile is P)."): hist[k] = states whose expansion discovered k new
 * states (ModelChecker.doNext's unseenSuccessorStates, Worker.setOutDegree),
 * *n = max k + 1.  Needs tlcg_opts.outdegree and TLC's first-discoverer
 * parents: a global-engine run in TLC order (world 1) or the component
 * engine; refused otherwise, and after tlcg_recover.  [TLC-ext] */
int tlcg_outdegree(tlcg_ctx* c, uint64_t* hist, int32_t cap, int32_t* n);
/* State expansions the last check's kernels made (*out): the component
 * engine counts, per pass, the states expanded for the components that finish
 * in it -- each state of each component for a per-lane kernel
 * (component_body.h, component_lane.h), each code state of a walk once for all
 * the walk's M x 64 components for the one-walk-per-wavefront kernel
 * (component_wave.h); the component tree counts each component's states
 * (tree_body.h) or each walk's code states (tree_wave.h) of its last
 * successful pass; the one-rank global engine reports the states of its
 * expanded levels.  So distinct / expansions is 1 for a per-state kernel and
 * the components per walk for the wave kernels.  -2 for other engines.  (TLC
 * has no counterpart: its workers expand each state once.) */
int tlcg_expansions(tlcg_ctx* c, uint64_t* out);
/* States generated per BFS level: out[0] = the initial states, out[k] = the
 * successors generated by expanding level k - 1 (stutters included), *n =
 * expanded levels + 1.  The sum is tlcg_stats.generated; the sum of
 * out[0..E] is the count at the end of level E (what combining ranks that
 * stopped at different levels needs, tlcg_run_node / dist.py).  Refused after
 * tlcg_recover (the checkpoint holds only the total). */
int tlcg_level_generated(tlcg_ctx* c, uint64_t* out, int32_t cap, int32_t* n);
/* Successor ordinal bits (to split a parent_ref). */
int tlcg_ordinal_bits(const tlcg_model* m);
int tlcg_action_of_ordinal(const tlcg_model* m, int32_t ordinal);

/* TLC value syntax of a packed state, "/\ var = value" lines in declaration
 * order (compaction.tla:57-70).  Host only.  Returns length or <0. */
int tlcg_decode(const tlcg_model* m, uint64_t state, char* buf, int32_t cap);
/* Host-side reference semantics of the packed encoding (same code the
 * kernels run): initial state idx, and the successors of a state in Next
 * order.  Returns the successor count, or <0 on an evaluation error. */
uint64_t tlcg_host_init_state(const tlcg_model* m, uint64_t idx);
int tlcg_host_successors(const tlcg_model* m, uint64_t state, uint64_t* out, int32_t* actions, int32_t cap);
/* First failing invariant of a state: -1 all hold, else (index << 1) | is_error. */
int tlcg_host_check_invariants(const tlcg_model* m, uint64_t state);
/* the same for either width */
int tlcg_decode_words(const tlcg_model* m, const uint64_t* state, char* buf, int32_t cap);
int tlcg_host_init_state_words(const tlcg_model* m, uint64_t idx, uint64_t* out);
int tlcg_host_successors_words(const tlcg_model* m, const uint64_t* state, uint64_t* out, int32_t* actions,
                               int32_t cap);
int tlcg_host_check_invariants_words(const tlcg_model* m, const uint64_t* state);
/* The same for n states (tlcg_state_words words each) into out[i]: one model
 * build (and user-invariant compile) for the batch.  0, or -2 on a bad model. */
int tlcg_host_check_invariants_batch(const tlcg_model* m, const uint64_t* states, uint64_t n, int32_t* out);
/* Self-check of the component engine's specialized evaluators against the
 * generic ones on the components of initial states [first, first + n), host
 * only.  Returns the states compared (0: the component engine does not take
 * this model), or < 0 on a disagreement. */
int64_t tlcg_host_component_selfcheck(const tlcg_model* m, uint64_t first, uint64_t n);
/* The component tree's closed-mode FPSet on the component of initial state
 * `comp`, replayed on the host with the engine's slot hash (the tuned
 * multiplier and the perfect-hash displacement table built from component
 * 0): out[0] = insert calls, out[1] = probe trips (each call's longest lane)
 * with the table, out[2] = without it; out[1] == out[0] when every insert
 * takes one CAS.  Host only: 0, -1 when the closed tree does not take the
 * component, -2 on a bad model. */
int tlcg_host_tree_slot_probes(const tlcg_model* m, uint64_t comp, int64_t* out);
/* PROPERTY Termination (compaction.tla:303-307).  Spec has no fairness, so a
 * behavior may stutter forever in its initial state: <>P fails iff an
 * initial state violates P.  Returns the first such initial state (TLC Init
 * order; the counterexample is that state followed by stuttering), -1 when
 * the property holds, < -1 on a bad model. */
int64_t tlcg_host_termination_counterexample(const tlcg_model* m);
/* ---- liveness: PROPERTY Termination (compaction.tla:303-307) on the GPU ----
 * <- TLC's liveness checker (tlc2.tool.liveness.LiveCheck / LiveWorker) for
 * Termination == <>P, P the guard of Terminating (compaction.tla:205-214).
 * The check walks G' = the states reachable from Init through not-P states
 * (the consistent part of the product with the tableau of []~P):
 *   TLCG_FAIR_NONE     Spec (compaction.tla:233): every behavior may stutter
 *                      forever, so <>P fails iff G' is not empty;
 *   TLCG_FAIR_WF_NEXT  Spec /\ WF_vars(Next) (SF_vars(Next) is the same
 *                      check): <>P fails iff G' holds a state where
 *                      <<Next>>_vars is disabled (TLCG_LIVE_STUTTERING) or a
 *                      cycle of non-stuttering steps (TLCG_LIVE_CYCLE, found by
 *                      peeling G' in Kahn order on the GPU).
 * The counterexample goes to states[0..*len) (tlcg_state_words uint64s
 * each) with the actions into them (TLCG_ACT_INIT first); it ends stuttering
 * (loop_to = -1) or steps back to states[loop_to] by back_action.  Which of
 * several counterexamples TLC prints is [TLC-ext]: this returns, without
 * fairness, the first not-P initial state in Init order; with fairness, the
 * least packed state of the shallowest level holding a stuck state, or the
 * first cycle reached from the shallowest state left after peeling.  The check
 * allocates its own device buffers (o->state_capacity and
 * o->log2_fpset_slots size them, grown on demand; o->device). */
enum { TLCG_FAIR_NONE = 0, TLCG_FAIR_WF_NEXT = 1 };
enum { TLCG_LIVE_HOLDS = 0, TLCG_LIVE_STUTTERING = 1, TLCG_LIVE_CYCLE = 2 };
typedef struct tlcg_liveness {
  int32_t holds;          /* 1: every behavior (fair behavior) reaches P */
  int32_t kind;           /* TLCG_LIVE_* */
  int32_t fairness;       /* TLCG_FAIR_* checked */
  int32_t depth;          /* BFS levels of G' */
  uint64_t states_notp;   /* |G'| */
  uint64_t init_notp;     /* initial states in G' */
  uint64_t edges_notp;    /* non-stuttering transitions into states of G' (from states of G') */
  uint64_t stuck;         /* states of G' where a (fair) behavior may stutter forever */
  uint64_t on_cycles;     /* states of G' left after peeling: on a cycle or reachable from one */
  uint64_t peel_rounds;   /* Kahn rounds */
  int32_t trace_len;      /* states in the counterexample (0 when it holds) */
  int32_t loop_to;        /* -1: the counterexample ends stuttering; else its back-edge target */
  int32_t back_action;    /* TLCG_ACT_* of the back edge (loop_to >= 0) */
  int32_t reserved;
  double kernel_ms;       /* device time of the BFS and peeling kernels (HIP events) */
  double wall_ms;         /* whole call */
} tlcg_liveness;
int tlcg_check_termination(const tlcg_model* m, const tlcg_opts* o, int32_t fairness, tlcg_liveness* out,
                           uint64_t* states, int32_t* actions, int32_t cap, int32_t* len, char* err,
                           int32_t err_cap);

/* Enable xGMI peer access among devices 0..n-1 (one process driving contexts
 * on several devices, e.g. tlc-hip -gpus N).  Returns the pairs enabled. */
int tlcg_peer_access(int32_t n);
/* HIP devices visible to this process (0 without a GPU). */
int tlcg_device_count(void);
/* Owner rank of a state under the context's partition. */
int tlcg_owner(tlcg_ctx* c, uint64_t state);

/* ---- partitioned (multi-rank) level, world > 1 ----
 * tlcg_init, then per level: tlcg_expand -> exchange outboxes (e.g. RCCL
 * all-to-all) -> tlcg_inbox + copy -> tlcg_absorb -> tlcg_end_level.
 * Records are 16 bytes: {uint64 state, uint64 parent_ref}.  A rank that is
 * no longer running (stats.status != TLCG_RUNNING -- e.g. an on-chip engine,
 * which completes the rank's share inside tlcg_init) returns 0 and its stats
 * from every call of the loop, with no records; a driver loops on the
 * combined termination as usual. */
int tlcg_expand(tlcg_ctx* c, tlcg_stats* st);
int tlcg_outbox(tlcg_ctx* c, int32_t dst, void** dev_records, uint64_t* n_records);
int tlcg_inbox(tlcg_ctx* c, uint64_t n_records, void** dev_records);
int tlcg_absorb(tlcg_ctx* c, uint64_t n_records, tlcg_stats* st);
int tlcg_end_level(tlcg_ctx* c, tlcg_stats* st);
/* Stream-ordered forms of the exchange copies: the first n records for dst
 * copied to caller memory (host or device), and the caller's n records (host
 * or device) copied in and absorbed.  The raw tlcg_outbox/tlcg_inbox pointers
 * need the caller to order its own copies against the context's stream. */
int tlcg_outbox_read(tlcg_ctx* c, int32_t dst, void* out, uint64_t n);
/* All destinations' records in rank order, contiguous (the all-to-all send
 * buffer; sum of the tlcg_outbox counts x 16 bytes), one stream sync. */
int tlcg_outbox_gather(tlcg_ctx* c, void* out);
int tlcg_absorb_records(tlcg_ctx* c, const void* records, uint64_t n, tlcg_stats* st);
/* The exchange when one process drives every rank (ctxs[r] = rank r of n, on
 * devices with peer access, tlcg_peer_access): after tlcg_expand on all of
 * them, copies each outbox into its owner's inbox device-to-device (source-
 * rank-major, as an all-to-all delivers) and waits for the copies.  n_in[d] =
 * records for tlcg_absorb(ctxs[d], n_in[d], ...).  Replaces distributed
 * TLC's FPSetManager.putBlock round trips within one node. */
int tlcg_exchange_local(tlcg_ctx* const* ctxs, int32_t n, uint64_t* n_in);
/* 1 when no successor leaves its rank (partition by an immutable `messages`):
 * each rank then runs tlcg_run alone and only the counts are combined. */
int tlcg_partition_closed(const tlcg_ctx* c);
/* The whole check by one process on the node's GPUs (tlc-hip -gpus N): n
 * ranks, rank r on device r mod tlcg_device_count(), each driven from its own
 * host thread through the level loop of tlcg_run_comm.  The records move over
 * RCCL (ncclCommInitAll) when every rank has a device of its own, else by
 * device-to-device copies between threads (TLCG_NODE_TRANSPORT=local|rccl
 * forces one; st->transport says which ran).  *st gets the combined verdict
 * (the first error by level then rank, every rank's counts cut at the end of
 * its level; level sizes summed into levels[0..cap), *n_levels).  The
 * contexts are destroyed before return (tlcg_run_node_trace also returns the
 * counterexample; TLC's own -workers 1 trace is re-derived on one GPU). */
int tlcg_run_node(const tlcg_model* m, const tlcg_opts* o, int32_t n, tlcg_stats* st, uint64_t* levels,
                  int32_t cap, int32_t* n_levels, char* err, int32_t err_cap);
/* tlcg_run_node plus the first error's counterexample without a re-run
 * (SURVEY 8(e)): the parent references walked across the ranks' stores,
 * host-mediated (each hop's owner reads the state, the transport hands it to
 * every rank).  states[i * words ..] (tlcg_state_words) and actions[i]
 * (TLCG_ACT_*, TLCG_ACT_INIT for the first) for i < min(*trace_len,
 * trace_cap); *trace_len = 0 when the model holds.  A shortest
 * counterexample; TLC -workers 1's own one needs TLC order on one GPU. */
int tlcg_run_node_trace(const tlcg_model* m, const tlcg_opts* o, int32_t n, tlcg_stats* st, uint64_t* levels,
                        int32_t cap, int32_t* n_levels, uint64_t* states, int32_t* actions, int32_t trace_cap,
                        int32_t* trace_len, char* err, int32_t err_cap);
/* The same with the node's ranks kept across checks: tlcg_node_create builds
 * the n contexts and their transport once, tlcg_node_run runs one whole check
 * (the arguments and results of tlcg_run_node_trace) and may be called again;
 * tlcg_node_destroy frees them.  A check then costs its level loop only (a
 * context's FPSet shard and store are sized by the first check and reused,
 * as a TLC server's FPSet outlives one exploration).  One thread of the
 * caller at a time per node. */
typedef struct tlcg_node tlcg_node;
int tlcg_node_create(const tlcg_model* m, const tlcg_opts* o, int32_t n, tlcg_node** out, char* err,
                     int32_t err_cap);
int tlcg_node_run(tlcg_node* node, tlcg_stats* st, uint64_t* levels, int32_t cap, int32_t* n_levels,
                  uint64_t* states, int32_t* actions, int32_t trace_cap, int32_t* trace_len, char* err,
                  int32_t err_cap);
void tlcg_node_destroy(tlcg_node* node);

/* ---- one process per GPU over RCCL (xGMI) ----
 * Rank 0 calls tlcg_comm_unique_id and hands the 128 bytes to every rank (the
 * caller's own channel, e.g. a torch.distributed broadcast); every rank
 * creates its context (tlcg_opts.rank / world) and calls tlcg_comm_init with
 * them; then tlcg_run_comm runs the whole check on all ranks: a closed
 * partition runs each rank alone, an open one runs every BFS level as
 * expand -> ncclAllGather of the per-destination counts -> grouped
 * ncclSend/ncclRecv of the 16-B records -> absorb, with an ncclAllReduce
 * deciding termination.  *st and levels[0..*n_levels) are the combined result
 * (the same on every rank; the first error by level, then rank, with every
 * rank's counts cut at the end of its level); on an error every rank's
 * tlcg_trace_words then returns the counterexample walked across the ranks'
 * stores (tlcg_run_node_trace).  A collective that does not
 * complete within TLCG_COMM_TIMEOUT_S seconds (default 600) aborts the
 * communicator and returns an error.  RCCL is loaded at run time
 * (librccl.so.1); tlcg_comm_available says whether it can be. */
int tlcg_comm_available(void);
int tlcg_comm_unique_id(void* id, int32_t cap);
int tlcg_comm_init(tlcg_ctx* c, const void* id, int32_t len);
/* The rank count of the context's RCCL communicator (ncclCommCount), 0 when
 * it has none: what a caller reports as the ranks the exchange really ran on. */
int tlcg_comm_size(tlcg_ctx* c);
int tlcg_run_comm(tlcg_ctx* c, tlcg_stats* st, uint64_t* levels, int32_t cap, int32_t* n_levels);

/* TLC -checkpoint: write the run's committed levels (state store + parent
 * log, level sizes, counters) to `path` between levels of a global-engine
 * run (the component engine finishes inside tlcg_init). */
int tlcg_checkpoint(tlcg_ctx* c, const char* path);
/* TLC -recover: resume from a checkpoint taken with the same constants and
 * options; the FPSet is rebuilt from the stored states.  Then call
 * tlcg_step_level (or the partitioned level calls) as after tlcg_init. */
int tlcg_recover(tlcg_ctx* c, const char* path, tlcg_stats* st);

/* Diagnostic: compile the kernels specialized for these constants (hipRTC)
 * for `arch` without a device (with user invariants: also the global engine's
 * user-check module); returns the code-object bytes or <0 (err). */
int tlcg_jit_selftest(const tlcg_model* m, const char* arch, char* err, int32_t cap);

/* HIP stream (hipStream_t) the context launches on, for event timing. */
void* tlcg_stream(tlcg_ctx* c);

#ifdef __cplusplus
}
#endif
#endif /* TLCGPU_H */
