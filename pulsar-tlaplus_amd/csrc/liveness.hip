// pulsar-tlaplus_amd/csrc/liveness.hip -- PROPERTY Termination on the GPU:
// TLC's liveness check (tlc2.tool.liveness) of <>P, compaction.tla:303-307,
// over the spec's state graph.
//
// P is the guard of Terminating (terminating_enabled, compaction.tla:205-214
// and :304-307 are the same conjunction).  A behavior violates <>P iff it
// never reaches a P state, so every counterexample lives in G', the states
// reachable from Init through not-P states only.  (TLC builds the product of
// the state graph with the tableau of the negated property, []~P; its
// consistent part is exactly G'.)  Fairness decides which infinite paths of
// G' are behaviors:
//   - none (Spec, compaction.tla:233): a behavior may stutter forever, so
//     every state of G' ends a counterexample; the shortest is the first
//     not-P initial state followed by stuttering;
//   - WF_vars(Next) (or SF_vars(Next): <<Next>>_vars is enabled in a state or
//     not, so the two agree here): a fair behavior stutters forever only where
//     <<Next>>_vars is disabled -- a state all of whose successors equal it
//     ("stuck") -- and otherwise takes infinitely many non-stuttering steps.
//     <>P fails iff G' holds a stuck state or a cycle of non-stuttering steps.
//
// The GPU pass:
//   1. BFS over G' (k_lv_init, k_lv_expand per level): successors that
//      satisfy P end the path and are not stored; the others go through an
//      HBM FPSet (kernels.h fpset_put) into a level-ordered store with parent
//      references, exactly like the safety engine's, and every edge into a
//      not-P state adds 1 to that state's in-degree (indexed by FPSet slot, so
//      no index lookup is needed while the level is being built).  A state
//      with no non-stuttering successor is flagged stuck.
//   2. Cycle test by Kahn peeling (k_lv_zero, k_lv_peel): repeatedly remove
//      the states of in-degree 0 and decrement their successors; G' is
//      acyclic iff every state is removed.
//   3. Counterexample: the shallowest stuck state (least packed word among
//      the stuck states of the shallowest level) and its BFS path from Init;
//      or, for a cycle, the states left after peeling are copied to the host,
//      peeled again from the other side (states with no successor left), and
//      walked from the shallowest one until a state repeats: the lasso is the
//      BFS path to the repeated state plus the cycle back to it.
// Counterexample choice and the output text are [TLC-ext] (TLC picks its
// own); holds / fails, |G'|, its edge count and the shallowest stuck depth are
// cross-checked with the oracle's Tarjan SCC restatement (oracle/tlc_oracle.c
// -liveness).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

#include "host_model.h"
#include "kernels.h"
#include "tlcgpu.h"

using namespace tlcg;

namespace {

using u32 = uint32_t;
constexpr int LV_BLOCK = 256;

enum LvFlag { LV_FPSET = 1, LV_STORE = 2, LV_EVAL = 4, LV_LOOKUP = 8 };

struct LvCtr {
  unsigned long long n;      // states of G' stored
  unsigned long long edges;  // non-stuttering edges into not-P states
  unsigned long long stuck;  // stuck states of the level just expanded
  unsigned long long next;   // entries appended to the next peel list
  unsigned long long key_hi, key_lo, pick;  // least stuck state of a level, then its index
  unsigned long long first_init;            // Init index of the first not-P initial state
  unsigned int flags;
  unsigned int pad;
};

template <typename W>
struct LvBufs {
  Layout L;
  u64* slots;     // FPSet, 2^log2 slots (8 B, or 16 B wide)
  int log2;
  W* store;       // states of G' in BFS order
  u64* parent;    // parent_gidx << ord_bits | ordinal, NO_PARENT for initial states
  u32* slot_of;   // FPSet slot of each stored state
  u32* gidx_of;   // stored index of the state in each FPSet slot
  u32* indeg;     // per FPSet slot: edges from states of G'
  unsigned char* stuck;  // per state: fairness lets a behavior stutter here forever
  u64 cap;        // store capacity
  LvCtr* ctr;
};

// Block-aggregated claim of indices in a global counter: one atomic per
// block per call instead of one per wave (a single counter serializes its
// atomics).  Every thread of the block calls it (uniform control flow) with
// NP predicates; at[j] gets the index of each true one, in (wave, j, lane)
// order.
template <int NP>
__device__ __forceinline__ void block_claim(const bool* pred, u64* at, unsigned long long* ctr) {
  __shared__ unsigned s_wcnt[LV_BLOCK / 64];
  __shared__ unsigned long long s_base;
  const int w = (int)(threadIdx.x >> 6);
  u64 m[NP];
  unsigned tot = 0;
#pragma unroll
  for (int j = 0; j < NP; ++j) {
    m[j] = __ballot(pred[j]);
    tot += (unsigned)__popcll(m[j]);
  }
  if (__lane_id() == 0) s_wcnt[w] = tot;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned sum = 0;
    for (int i = 0; i < LV_BLOCK / 64; ++i) sum += s_wcnt[i];
    s_base = sum ? atomicAdd(ctr, (unsigned long long)sum) : 0ull;
  }
  __syncthreads();
  u64 base = s_base;
  for (int i = 0; i < w; ++i) base += s_wcnt[i];
#pragma unroll
  for (int j = 0; j < NP; ++j) {
    at[j] = base + (u64)__popcll(m[j] & lanemask_lt());
    base += (u64)__popcll(m[j]);
  }
  __syncthreads();  // (s_wcnt / s_base are reused by the next call)
}

template <typename W>
__host__ __device__ inline bool lv_p(const Layout& L, W s) {
  return terminating_enabled(L, s);
}

// Move k of s (k < moves_bound(L)): Producer's nkv successors (key outer,
// value inner), then the compactor disjunct, then BrokerCrash.  Returns 1 with
// *t / *ord set when that move exists and changes the state, 0 otherwise, 2 on
// an evaluation error.  Stutters (Consumer, Terminating) are never moves.
template <typename W>
__host__ __device__ inline int lv_move(const Layout& L, W s, int k, W* t, int* ord) {
  const int np = L.producer ? L.nkv : 0;
  if (k < np) {
    const int len = st_len(L, s);
    if (len >= L.N) return 0;
    *t = producer_succ(L, s, len, k);
    *ord = ordinal_of(L, ACT_PRODUCER, k);
    return *t != s;
  }
  int act = 0;
  if (k == np) {
    const int r = compactor_step(L, s, t, &act);
    if (r == 2) return 2;
    *ord = ordinal_of(L, act, 0);
    return r == 1 && *t != s;
  }
  if (!crash_step(L, s, t)) return 0;
  *ord = ordinal_of(L, ACT_CRASH, 0);
  return *t != s;
}
__host__ __device__ inline int moves_bound(const Layout& L) { return (L.producer ? L.nkv : 0) + 2; }

// FPSet lookup of a state known to be present (all inserts finished in an
// earlier launch, so plain loads see every slot).
template <typename W>
__device__ __forceinline__ u64 lv_lookup(const u64* slots, int log2, W t) {
  const u64 mask = (1ull << log2) - 1;
  u64 i = mixw<W>(t) >> (64 - log2);
  for (int p = 0; p < MAX_PROBE; ++p) {
    if constexpr (sizeof(W) == 8) {
      const u64 v = slots[i];
      if (v == ((u64)t | SLOT_TAG)) return i;
      if (v == 0) return ~0ull;
    } else {
      const u64 hi = slots[2 * i];
      if (hi == 0) return ~0ull;
      if ((hi & ~WIDE_READY) == ((u64)(t >> 64) | SLOT_TAG) && slots[2 * i + 1] == (u64)t) return i;
    }
    i = (i + 1) & mask;
  }
  return ~0ull;
}

// insert t (a not-P state) with parent reference pref; every thread of the
// block calls it (want = this lane has a state to insert)
template <typename W>
__device__ __forceinline__ void lv_insert(const LvBufs<W>& B, bool want, W t, u64 pref, bool edge) {
  u64 slot = 0;
  int r = 0;
  if (want) {
    r = fpset_put<W>(B.slots, B.log2, t, mixw<W>(t), &slot);
    if (r < 0) atomicOr(&B.ctr->flags, (unsigned)LV_FPSET);
    else if (edge) atomicAdd(&B.indeg[slot], 1u);
  }
  const bool fresh = want && r == 1;
  u64 g = 0;
  block_claim<1>(&fresh, &g, &B.ctr->n);
  if (fresh) {
    if (g >= B.cap) {
      atomicOr(&B.ctr->flags, (unsigned)LV_STORE);
    } else {
      B.store[g] = t;
      B.parent[g] = pref;
      B.slot_of[g] = (u32)slot;
      B.gidx_of[slot] = (u32)g;
    }
  }
}

// A batch of up to LV_BATCH candidates of one lane: their first FPSet slots
// are loaded together (and CASed together where empty), so a lane waits on
// one scattered round trip per batch instead of one per candidate; collisions
// go on probing (fpset_put_from).  Wide states take the wave-uniform
// two-word insert one by one.  slot[j] gets the candidate's slot, fresh[j]
// whether this lane inserted it.
constexpr int LV_BATCH = 4;
template <typename W>
__device__ __forceinline__ void lv_put_batch(const LvBufs<W>& B, const bool* want, const W* t, u64* slot,
                                             bool* fresh) {
  if constexpr (sizeof(W) == 8) {
    const int sh = 64 - B.log2;
    const u64 mask = (1ull << B.log2) - 1;
    u64 v[LV_BATCH];
#pragma unroll
    for (int j = 0; j < LV_BATCH; ++j) {
      slot[j] = mix64((u64)t[j]) >> sh;
      v[j] = want[j] ? __builtin_nontemporal_load(&B.slots[slot[j]]) : 1;
    }
#pragma unroll
    for (int j = 0; j < LV_BATCH; ++j)
      if (want[j] && v[j] == 0)
        v[j] = atomicCAS((unsigned long long*)&B.slots[slot[j]], 0ull, (unsigned long long)((u64)t[j] | SLOT_TAG));
#pragma unroll
    for (int j = 0; j < LV_BATCH; ++j) {
      fresh[j] = false;
      if (!want[j]) continue;
      const u64 key = (u64)t[j] | SLOT_TAG;
      if (v[j] == 0) {
        fresh[j] = true;
      } else if (v[j] != key) {
        const int r = fpset_put_from(B.slots, mask, key, (slot[j] + 1) & mask, &slot[j]);
        if (r < 0) {
          atomicOr(&B.ctr->flags, (unsigned)LV_FPSET);
          slot[j] = ~0ull;
        }
        fresh[j] = r == 1;
      }
    }
  } else {
#pragma unroll
    for (int j = 0; j < LV_BATCH; ++j) {
      fresh[j] = false;
      if (!want[j]) continue;
      const int r = fpset_put<W>(B.slots, B.log2, t[j], mixw<W>(t[j]), &slot[j]);
      if (r < 0) {
        atomicOr(&B.ctr->flags, (unsigned)LV_FPSET);
        slot[j] = ~0ull;
      }
      fresh[j] = r == 1;
    }
  }
}

// the same for lookups of states known to be present: first slots together
template <typename W>
__device__ __forceinline__ void lv_lookup_batch(const LvBufs<W>& B, const bool* want, const W* t, u64* slot) {
  if constexpr (sizeof(W) == 8) {
    const int sh = 64 - B.log2;
    const u64 mask = (1ull << B.log2) - 1;
    u64 v[LV_BATCH];
#pragma unroll
    for (int j = 0; j < LV_BATCH; ++j) {
      slot[j] = mix64((u64)t[j]) >> sh;
      v[j] = want[j] ? B.slots[slot[j]] : 0;
    }
#pragma unroll
    for (int j = 0; j < LV_BATCH; ++j) {
      if (!want[j]) continue;
      const u64 key = (u64)t[j] | SLOT_TAG;
      if (v[j] == key) continue;
      u64 i = slot[j];
      slot[j] = ~0ull;
      for (int p = 1; p < MAX_PROBE && v[j] != 0; ++p) {
        i = (i + 1) & mask;
        v[j] = B.slots[i];
        if (v[j] == key) {
          slot[j] = i;
          break;
        }
      }
    }
  } else {
#pragma unroll
    for (int j = 0; j < LV_BATCH; ++j) slot[j] = want[j] ? lv_lookup<W>(B.slots, B.log2, t[j]) : ~0ull;
  }
}

template <typename W>
__global__ __launch_bounds__(LV_BLOCK) void k_lv_init(LvBufs<W> B, u64 n_init) {
  const u64 stride = (u64)gridDim.x * LV_BLOCK;
  for (u64 base = (u64)blockIdx.x * LV_BLOCK; base < n_init; base += stride) {
    const u64 i = base + threadIdx.x;
    bool want = false;
    W s = 0;
    if (i < n_init) {
      s = init_state<W>(B.L, i);
      want = !lv_p(B.L, s);
    }
    // the first not-P initial state: the wave's lowest such index, one atomic per wave
    const u64 wm = __ballot(want);
    if (wm && __lane_id() == __ffsll((long long)wm) - 1) atomicMin(&B.ctr->first_init, (unsigned long long)i);
    lv_insert(B, want, s, NO_PARENT, false);
  }
}

// one BFS level of G': states [a, b)
template <typename W>
__global__ __launch_bounds__(LV_BLOCK) void k_lv_expand(LvBufs<W> B, u64 a, u64 b, int fair) {
  const Layout& L = B.L;
  const int kmax = moves_bound(L);
  const u64 stride = (u64)gridDim.x * LV_BLOCK;
  // edges and stuck states are summed in registers over the whole loop and
  // added once per wave at the end (atomics on one counter serialize)
  u64 edges = 0, nstuck = 0;
  bool err = false;
  for (u64 base = a + (u64)blockIdx.x * LV_BLOCK; base < b; base += stride) {
    const u64 g = base + threadIdx.x;
    const bool live = g < b;
    const W s = live ? B.store[g] : (W)0;
    int moves = 0;
    bool serr = false;
    for (int k0 = 0; k0 < kmax; k0 += LV_BATCH) {
      W t[LV_BATCH];
      int ord[LV_BATCH];
      bool want[LV_BATCH], fresh[LV_BATCH];
      u64 slot[LV_BATCH];
#pragma unroll
      for (int j = 0; j < LV_BATCH; ++j) {
        t[j] = 0;
        ord[j] = 0;
        const int r = live && k0 + j < kmax ? lv_move(L, s, k0 + j, &t[j], &ord[j]) : 0;
        serr |= r == 2;
        moves += r == 1;
        want[j] = r == 1 && !lv_p(L, t[j]);
        edges += want[j];
      }
      lv_put_batch(B, want, t, slot, fresh);
      u64 ats[LV_BATCH];
      block_claim<LV_BATCH>(fresh, ats, &B.ctr->n);
#pragma unroll
      for (int j = 0; j < LV_BATCH; ++j) {
        if (want[j] && slot[j] != ~0ull) atomicAdd(&B.indeg[slot[j]], 1u);
        const u64 at = ats[j];
        if (fresh[j]) {
          if (at >= B.cap) {
            atomicOr(&B.ctr->flags, (unsigned)LV_STORE);
          } else {
            B.store[at] = t[j];
            B.parent[at] = (g << L.ord_bits) | (u64)ord[j];
            B.slot_of[at] = (u32)slot[j];
            B.gidx_of[slot[j]] = (u32)at;
          }
        }
      }
    }
    err |= serr;
    const bool stuck = live && !serr && (fair == TLCG_FAIR_NONE || moves == 0);
    if (live) B.stuck[g] = stuck;
    nstuck += stuck;
  }
  if (err) atomicOr(&B.ctr->flags, (unsigned)LV_EVAL);
  const u64 e = wave_sum_u64(edges), sk = wave_sum_u64(nstuck);
  if (__lane_id() == 0) {
    if (e) atomicAdd(&B.ctr->edges, (unsigned long long)e);
    if (sk) atomicAdd(&B.ctr->stuck, (unsigned long long)sk);
  }
}

// the least stuck state of level [a, b): its high word, then its low word, then its index
template <typename W>
__global__ __launch_bounds__(LV_BLOCK) void k_lv_pick(LvBufs<W> B, u64 a, u64 b, int phase) {
  const u64 stride = (u64)gridDim.x * LV_BLOCK;
  for (u64 g = a + (u64)blockIdx.x * LV_BLOCK + threadIdx.x; g < b; g += stride) {
    if (!B.stuck[g]) continue;
    const W s = B.store[g];
    const u64 hi = sizeof(W) == 8 ? 0 : (u64)((unsigned __int128)s >> 64), lo = (u64)s;
    if (phase == 0) atomicMin(&B.ctr->key_hi, (unsigned long long)hi);
    else if (phase == 1) { if (hi == B.ctr->key_hi) atomicMin(&B.ctr->key_lo, (unsigned long long)lo); }
    else if (hi == B.ctr->key_hi && lo == B.ctr->key_lo) B.ctr->pick = g;
  }
}

// Kahn peeling: the states of in-degree 0 ...
template <typename W>
__global__ __launch_bounds__(LV_BLOCK) void k_lv_zero(LvBufs<W> B, u64 n, u32* list) {
  const u64 stride = (u64)gridDim.x * LV_BLOCK;
  for (u64 base = (u64)blockIdx.x * LV_BLOCK; base < n; base += stride) {
    const u64 g = base + threadIdx.x;
    const bool z = g < n && B.indeg[B.slot_of[g]] == 0;
    u64 at = 0;
    block_claim<1>(&z, &at, &B.ctr->next);
    if (z) list[at] = (u32)g;
  }
}

// ... then, per round, remove them: each successor in G' loses one in-edge,
// and the ones that reach 0 form the next round
template <typename W>
__global__ __launch_bounds__(LV_BLOCK) void k_lv_peel(LvBufs<W> B, const u32* list, u64 n, u32* next) {
  const Layout& L = B.L;
  const int kmax = moves_bound(L);
  const u64 stride = (u64)gridDim.x * LV_BLOCK;
  for (u64 base = (u64)blockIdx.x * LV_BLOCK; base < n; base += stride) {
    const u64 i = base + threadIdx.x;
    const bool live = i < n;
    const W s = live ? B.store[list[i]] : (W)0;
    for (int k0 = 0; k0 < kmax; k0 += LV_BATCH) {
      W t[LV_BATCH];
      bool want[LV_BATCH];
      u64 slot[LV_BATCH];
#pragma unroll
      for (int j = 0; j < LV_BATCH; ++j) {
        t[j] = 0;
        int ord = 0;
        want[j] = live && k0 + j < kmax && lv_move(L, s, k0 + j, &t[j], &ord) == 1 && !lv_p(L, t[j]);
      }
      lv_lookup_batch(B, want, t, slot);
      bool freed[LV_BATCH];
      u32 tg[LV_BATCH];
#pragma unroll
      for (int j = 0; j < LV_BATCH; ++j) {
        freed[j] = false;
        tg[j] = 0;
        if (want[j]) {
          if (slot[j] == ~0ull) {
            atomicOr(&B.ctr->flags, (unsigned)LV_LOOKUP);
          } else if (atomicSub(&B.indeg[slot[j]], 1u) == 1u) {
            freed[j] = true;
            tg[j] = B.gidx_of[slot[j]];
          }
        }
      }
      u64 ats[LV_BATCH];
      block_claim<LV_BATCH>(freed, ats, &B.ctr->next);
#pragma unroll
      for (int j = 0; j < LV_BATCH; ++j)
        if (freed[j]) next[ats[j]] = tg[j];
    }
  }
}

// the states left after peeling (on or after a cycle): their indices
template <typename W>
__global__ __launch_bounds__(LV_BLOCK) void k_lv_left(LvBufs<W> B, u64 n, u32* list) {
  const u64 stride = (u64)gridDim.x * LV_BLOCK;
  for (u64 base = (u64)blockIdx.x * LV_BLOCK; base < n; base += stride) {
    const u64 g = base + threadIdx.x;
    const bool z = g < n && B.indeg[B.slot_of[g]] != 0;
    u64 at = 0;
    block_claim<1>(&z, &at, &B.ctr->next);
    if (z) list[at] = (u32)g;
  }
}

unsigned grid_for(u64 n) {
  const u64 blocks = (n + LV_BLOCK - 1) / LV_BLOCK;
  return (unsigned)std::max<u64>(1, std::min<u64>(blocks, 256 * 32));
}

struct DevMem {
  std::vector<void*> ptrs;
  ~DevMem() {
    for (void* p : ptrs) hipFree(p);
  }
  template <typename T>
  bool alloc(T** p, u64 count) {
    *p = nullptr;
    if (hipMalloc((void**)p, std::max<u64>(count, 1) * sizeof(T)) != hipSuccess) return false;
    ptrs.push_back(*p);
    return true;
  }
};

#define LV_CHECK(x)                                                              \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      *err = std::string(#x ": ") + hipGetErrorString(e_);                       \
      return -4;                                                                 \
    }                                                                            \
  } while (0)

struct LvTrace {
  std::vector<u128> states;
  std::vector<int> actions;
  int loop_to = -1, back_action = -1;
};

// BFS path from Init to stored state g (states and the actions into them)
template <typename W>
int path_to(const LvBufs<W>& B, u64 g, LvTrace* tr, std::string* err) {
  std::vector<std::pair<W, u64>> rev;
  for (;;) {
    W s;
    u64 p;
    LV_CHECK(hipMemcpy(&s, B.store + g, sizeof(W), hipMemcpyDeviceToHost));
    LV_CHECK(hipMemcpy(&p, B.parent + g, sizeof(u64), hipMemcpyDeviceToHost));
    rev.push_back({s, p});
    if (p == NO_PARENT || rev.size() > 1u << 20) break;
    g = p >> B.L.ord_bits;
  }
  for (size_t i = rev.size(); i-- > 0;) {
    tr->states.push_back((u128)rev[i].first);
    const u64 p = rev[i].second;
    tr->actions.push_back(p == NO_PARENT ? TLCG_ACT_INIT
                                         : action_of_ordinal(B.L, (int)(p & ((1ull << B.L.ord_bits) - 1))));
  }
  return 0;
}

// Host: the states left after peeling (st, with their BFS indices idx,
// ascending) lie on cycles or after them.  Peel them from the other side
// (drop states none of whose successors is left) so that every remaining state
// has a successor among them, then walk from the shallowest remaining state,
// taking the first remaining successor in Next order, until a state repeats.
// The lasso: *g_entry (the repeated state's BFS index), the cycle's other
// states with the actions into them, and the action back to the entry.
template <typename W>
int lasso_walk(const Layout& L, const std::vector<W>& st, const std::vector<u32>& idx, u64* g_entry,
               std::vector<u128>* cyc, std::vector<int>* cyc_act, int* back_action, std::string* err) {
  const size_t n = st.size();
  std::vector<std::pair<W, u32>> by_state(n);
  for (size_t i = 0; i < n; ++i) by_state[i] = {st[i], (u32)i};
  std::sort(by_state.begin(), by_state.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
  auto find = [&](W t) -> long {
    auto it = std::lower_bound(by_state.begin(), by_state.end(), t,
                               [](const std::pair<W, u32>& a, W v) { return a.first < v; });
    return it != by_state.end() && it->first == t ? (long)it->second : -1;
  };
  const int kmax = moves_bound(L);
  std::vector<std::vector<std::pair<u32, int>>> succ(n);  // (state, ordinal) in Next order
  std::vector<std::vector<u32>> pred(n);
  for (size_t i = 0; i < n; ++i)
    for (int k = 0; k < kmax; ++k) {
      W t;
      int ord = 0;
      if (lv_move(L, st[i], k, &t, &ord) != 1 || lv_p(L, t)) continue;
      const long j = find(t);
      if (j < 0) continue;
      succ[i].push_back({(u32)j, ord});
      pred[j].push_back((u32)i);
    }
  std::vector<size_t> outc(n);
  std::vector<char> alive(n, 1);
  std::vector<u32> q;
  for (size_t i = 0; i < n; ++i)
    if ((outc[i] = succ[i].size()) == 0) q.push_back((u32)i);
  while (!q.empty()) {
    const u32 v = q.back();
    q.pop_back();
    alive[v] = 0;
    for (u32 p : pred[v])
      if (alive[p] && --outc[p] == 0) q.push_back(p);
  }
  size_t start = 0;
  while (start < n && !alive[start]) ++start;
  if (start == n) {
    *err = "liveness: peeling left states but no cycle among them";
    return -1;
  }
  std::vector<long> seen(n, -1);
  std::vector<u32> walk;
  std::vector<int> ords;
  u32 v = (u32)start;
  while (seen[v] < 0) {
    seen[v] = (long)walk.size();
    walk.push_back(v);
    const auto* nx = &succ[v][0];
    while (!alive[nx->first]) ++nx;  // one exists: v kept a live successor
    ords.push_back(nx->second);
    v = nx->first;
  }
  const size_t c0 = (size_t)seen[v];
  *g_entry = idx[walk[c0]];
  for (size_t i = c0 + 1; i < walk.size(); ++i) {
    cyc->push_back((u128)st[walk[i]]);
    cyc_act->push_back(action_of_ordinal(L, ords[i - 1]));
  }
  *back_action = action_of_ordinal(L, ords.back());
  return 0;
}

template <typename W>
int run_liveness(const HostModel& hm, const tlcg_opts* o, int fair, tlcg_liveness* out, LvTrace* tr, std::string* err) {
  const Layout& L = hm.L;
  u64 cap = o && o->state_capacity ? o->state_capacity : (u64)1 << 22;
  int log2 = o && o->log2_fpset_slots > 0 ? o->log2_fpset_slots : 0;
  hipEvent_t e0, e1;
  LV_CHECK(hipEventCreate(&e0));
  LV_CHECK(hipEventCreate(&e1));
  struct EvGuard {
    hipEvent_t a, b;
    ~EvGuard() {
      hipEventDestroy(a);
      hipEventDestroy(b);
    }
  } evg{e0, e1};
  for (int attempt = 0;; ++attempt) {
    if (cap >= (1ull << 32) - 1) {
      *err = "the liveness check indexes states with 32 bits: more than 2^32 - 1 not-P states";
      return -5;
    }
    int lg = log2;
    if (lg <= 0 || attempt > 0) {
      lg = 10;
      while ((1ull << lg) < 2 * cap) ++lg;
    }
    if (lg > 32) lg = 32;
    DevMem mem;
    LvBufs<W> B;
    B.L = L;
    B.log2 = lg;
    B.cap = cap;
    const u64 nslots = 1ull << lg;
    if (!mem.alloc(&B.slots, nslots * (sizeof(W) / 8)) || !mem.alloc(&B.store, cap) || !mem.alloc(&B.parent, cap) ||
        !mem.alloc(&B.slot_of, cap) || !mem.alloc(&B.gidx_of, nslots) || !mem.alloc(&B.indeg, nslots) ||
        !mem.alloc(&B.stuck, cap) || !mem.alloc(&B.ctr, 1)) {
      if (cap > (1ull << 20) && attempt < 8) {
        // what HBM holds beside the caller's other buffers: a smaller start,
        // grown x4 below only if G' needs it
        cap /= 2;
        log2 = 0;
        continue;
      }
      *err = "liveness: device allocation failed (" + std::to_string(cap) + " states, 2^" + std::to_string(lg) +
             " FPSet slots)";
      return -5;
    }
    LV_CHECK(hipMemset(B.slots, 0, nslots * sizeof(W)));
    LV_CHECK(hipMemset(B.indeg, 0, nslots * sizeof(u32)));
    LvCtr h{};
    h.first_init = ~0ull;
    LV_CHECK(hipMemcpy(B.ctr, &h, sizeof h, hipMemcpyHostToDevice));
    auto read_ctr = [&]() -> int {
      LV_CHECK(hipMemcpy(&h, B.ctr, sizeof h, hipMemcpyDeviceToHost));
      return 0;
    };
    auto grow = [&]() {
      return (h.flags & (LV_FPSET | LV_STORE)) != 0;
    };
    float ms_total = 0.f, ms = 0.f;
    LV_CHECK(hipEventRecord(e0, 0));
    k_lv_init<W><<<grid_for(hm.n_init), LV_BLOCK>>>(B, hm.n_init);
    LV_CHECK(hipGetLastError());
    if (read_ctr()) return -4;
    std::vector<u64> level_base{0, std::min<u64>(h.n, cap)}, level_stuck;
    bool again = grow();
    while (!again && level_base.back() > level_base[level_base.size() - 2]) {
      const u64 a = level_base[level_base.size() - 2], b = level_base.back();
      LV_CHECK(hipMemset(&B.ctr->stuck, 0, sizeof(unsigned long long)));
      k_lv_expand<W><<<grid_for(b - a), LV_BLOCK>>>(B, a, b, fair);
      LV_CHECK(hipGetLastError());
      if (read_ctr()) return -4;
      if (h.flags & LV_EVAL) {
        *err = "liveness: an evaluation error while computing a successor (run the safety check first)";
        return -6;
      }
      if ((again = grow())) break;
      level_stuck.push_back(h.stuck);
      level_base.push_back(h.n);
    }
    LV_CHECK(hipEventRecord(e1, 0));
    LV_CHECK(hipEventSynchronize(e1));
    LV_CHECK(hipEventElapsedTime(&ms, e0, e1));
    ms_total += ms;
    if (again) {
      cap *= 4;
      continue;  // redo with a larger store and FPSet
    }
    const u64 n = h.n;
    out->states_notp = n;
    out->init_notp = level_base[1];
    out->edges_notp = h.edges;
    out->depth = (int32_t)(level_base.size() - 2 + (n > 0 ? 1 : 0));
    out->stuck = 0;
    for (u64 x : level_stuck) out->stuck += x;
    // 2. Kahn peeling
    u32 *la = nullptr, *lb = nullptr;
    if (!mem.alloc(&la, n) || !mem.alloc(&lb, n)) {
      *err = "liveness: device allocation failed (peel lists)";
      return -5;
    }
    LV_CHECK(hipEventRecord(e0, 0));
    LV_CHECK(hipMemset(&B.ctr->next, 0, sizeof(unsigned long long)));
    k_lv_zero<W><<<grid_for(n), LV_BLOCK>>>(B, n, la);
    LV_CHECK(hipGetLastError());
    if (read_ctr()) return -4;
    u64 removed = 0, cur = h.next;
    int rounds = 0;
    while (cur) {
      removed += cur;
      ++rounds;
      LV_CHECK(hipMemset(&B.ctr->next, 0, sizeof(unsigned long long)));
      k_lv_peel<W><<<grid_for(cur), LV_BLOCK>>>(B, la, cur, lb);
      LV_CHECK(hipGetLastError());
      if (read_ctr()) return -4;
      if (h.flags & LV_LOOKUP) {
        *err = "liveness: a successor in G' is missing from the FPSet";
        return -6;
      }
      cur = h.next;
      std::swap(la, lb);
    }
    LV_CHECK(hipEventRecord(e1, 0));
    LV_CHECK(hipEventSynchronize(e1));
    LV_CHECK(hipEventElapsedTime(&ms, e0, e1));
    ms_total += ms;
    out->peel_rounds = rounds;
    out->on_cycles = n - removed;
    out->kernel_ms = ms_total;
    // 3. verdict and counterexample
    if (out->stuck && fair == TLCG_FAIR_NONE) {
      // every state of G' may stutter forever: the shortest counterexample is
      // the first not-P initial state in Init order, then stuttering
      out->holds = 0;
      out->kind = TLCG_LIVE_STUTTERING;
      tr->states.push_back((u128)init_state<W>(L, h.first_init));
      tr->actions.push_back(TLCG_ACT_INIT);
      return 0;
    }
    if (out->stuck) {
      out->holds = 0;
      out->kind = TLCG_LIVE_STUTTERING;
      size_t lv = 0;
      while (level_stuck[lv] == 0) ++lv;
      const u64 a = level_base[lv], b = level_base[lv + 1];
      h.key_hi = h.key_lo = ~0ull;
      h.pick = ~0ull;
      LV_CHECK(hipMemcpy(B.ctr, &h, sizeof h, hipMemcpyHostToDevice));
      for (int ph = 0; ph < 3; ++ph) k_lv_pick<W><<<grid_for(b - a), LV_BLOCK>>>(B, a, b, ph);
      LV_CHECK(hipGetLastError());
      if (read_ctr()) return -4;
      if (h.pick == ~0ull) {
        *err = "liveness: no stuck state found in its level";
        return -6;
      }
      return path_to(B, h.pick, tr, err);
    }
    if (removed == n) {
      out->holds = 1;
      out->kind = TLCG_LIVE_HOLDS;
      return 0;
    }
    // a cycle: copy the states left after peeling to the host
    out->holds = 0;
    out->kind = TLCG_LIVE_CYCLE;
    const u64 left = n - removed;
    if (left > (1ull << 26)) {
      *err = "liveness: " + std::to_string(left) + " states lie on or after cycles; the lasso extraction takes at most 2^26";
      return -5;
    }
    LV_CHECK(hipMemset(&B.ctr->next, 0, sizeof(unsigned long long)));
    k_lv_left<W><<<grid_for(n), LV_BLOCK>>>(B, n, la);
    LV_CHECK(hipGetLastError());
    std::vector<u32> idx(left);
    std::vector<W> st(left);
    LV_CHECK(hipMemcpy(idx.data(), la, left * sizeof(u32), hipMemcpyDeviceToHost));
    std::sort(idx.begin(), idx.end());
    for (u64 i = 0; i < left; ++i) LV_CHECK(hipMemcpy(&st[i], B.store + idx[i], sizeof(W), hipMemcpyDeviceToHost));
    u64 g_entry = 0;
    std::vector<u128> cyc;
    std::vector<int> cyc_act;
    int back = -1;
    if (lasso_walk(L, st, idx, &g_entry, &cyc, &cyc_act, &back, err) != 0) return -6;
    // the BFS path to the cycle's entry, then around the cycle back to it
    if (path_to(B, g_entry, tr, err)) return -4;
    tr->loop_to = (int)tr->states.size() - 1;
    tr->states.insert(tr->states.end(), cyc.begin(), cyc.end());
    tr->actions.insert(tr->actions.end(), cyc_act.begin(), cyc_act.end());
    tr->back_action = back;
    return 0;
  }
}

}  // namespace

extern "C" int tlcg_check_termination(const tlcg_model* m, const tlcg_opts* o, int32_t fairness, tlcg_liveness* out,
                                      uint64_t* states, int32_t* actions, int32_t cap, int32_t* len, char* err,
                                      int32_t err_cap) {
  auto fail = [&](int rc, const std::string& e) {
    if (err && err_cap > 0) std::snprintf(err, (size_t)err_cap, "%s", e.c_str());
    return rc;
  };
  if (!m || !out) return fail(-1, "null argument");
  if (fairness != TLCG_FAIR_NONE && fairness != TLCG_FAIR_WF_NEXT) return fail(-1, "unknown fairness");
  std::memset(out, 0, sizeof *out);
  out->fairness = fairness;
  if (len) *len = 0;
  HostModel hm;
  std::string e;
  if (!build_model(*m, &hm, &e)) return fail(-3, e);
  if (hipSetDevice(o ? o->device : 0) != hipSuccess) return fail(-4, "hipSetDevice failed");
  const auto t0 = std::chrono::steady_clock::now();
  LvTrace tr;
  const int words = state_words(hm.L);
  const int rc = words == 1 ? run_liveness<u64>(hm, o, fairness, out, &tr, &e)
                            : run_liveness<u128>(hm, o, fairness, out, &tr, &e);
  out->wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  if (rc) return fail(rc, e);
  out->trace_len = (int32_t)tr.states.size();
  out->loop_to = tr.loop_to;
  out->back_action = tr.back_action;
  if (states && actions && len) {
    const int32_t n = std::min<int32_t>(cap, out->trace_len);
    for (int32_t i = 0; i < n; ++i) {
      split_words(tr.states[i], states + (size_t)i * words, words);
      actions[i] = tr.actions[i];
    }
    *len = n;
  }
  return 0;
}
