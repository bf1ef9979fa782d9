// pulsar-tlaplus_amd/csrc/tlcgpu.hip -- the gfx950 BFS level kernels and the
// host runtime behind include/tlcgpu.h.
//
// One BFS level = one `k_expand` launch over the frontier (a contiguous slice
// of the resident state store).  Per parent state the kernel evaluates the
// Next disjuncts (compaction.tla:216-231) on the packed word, counts every
// successor as generated, inserts non-stuttering successors into the HBM
// FPSet with a 64-bit CAS, checks invariants on the new ones, and appends them
// (wave ballot -> LDS stage -> one global atomic per block chunk) to the next
// level together with a parent-pointer entry for traces.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>
#include <chrono>
#include <thread>
#include <type_traits>
#include <sys/mman.h>

#include "component.h"
#include "component_body.h"  // (CodeShape: the code pass's FPSet size)
#include "component_code.h"
#include "tree.h"
#include "exchange.h"
#include "host_model.h"
#include "jit.h"
#include "kernels.h"
#include "tlcgpu.h"

using namespace tlcg;

namespace {

struct ExpandArgs {
  Layout L;
  const u64* frontier;
  u64 n_front;
  u64 front_gidx0;  // gidx of frontier[0]
  u64* slots;
  int log2;
  u64* states_out;  // next level (store + level_base[d+1])
  u64* parents_out;
  u64 cap_out;      // room for new states
  u64* slot_out;    // TLC order: FPSet slot of every new state
  u64* dkey_slot;   // TLC order: min discovery key per FPSet slot
  LevelCtr* ctr;
  u64 rank_tag;     // rank << 56
  int rank, world;
  u64 owner_mask;
  u64* outbox;      // world > 1: [world][outbox_cap] records {state, parent_ref}
  u64 outbox_cap;
};

// owner rank of a state: wide states are only partitioned by `messages`,
// which then lies in the low word (tlcg_create checks).  The LOW 32 bits of
// the mix pick the owner: FPSet slots come from its high bits, and with the
// whole state as the partition key (partition 2) an owner taken from the high
// bits would leave every rank's states in 1/world of its table.
TLCG_HD int owner_hash(u64 key, int world) { return (int)(((mix64(key) & 0xFFFFFFFFull) * (u64)world) >> 32); }
template <typename W>
__device__ __forceinline__ int owner_of(W s, u64 owner_mask, int world) {
  return owner_hash((u64)s & owner_mask, world);
}

// overflow flag of a failed FPSet insert
__device__ __forceinline__ unsigned ovf_of(int r) { return r == -2 ? (unsigned)OVF_WIDE_SPIN : (unsigned)OVF_FPSET; }

// ---- user invariants (user_inv.h): every invariant of the cfg, in its
// order, on each state of a new level (the expand kernels check none when the
// cfg has user invariants, Layout.defer_inv).  The event key is the state's
// first-discovery key -- its parent reference without the rank, or its Init
// index on level 0 -- as the expand kernels' (kernels.h make_event), so the
// least event of a level is TLC's first error there in TLC-order mode.
// (kernels.h user_check_body is the hipRTC kernel; this one interprets the
// program, for TLCG_JIT=0 or a failed hipRTC build)
template <typename W>
__global__ __launch_bounds__(BLOCK) void k_user_check(Layout L, const UserProg* __restrict__ P, UserCheckArgs a) {
  const u64 i = (u64)blockIdx.x * BLOCK + threadIdx.x;
  if (i >= a.n) return;
  const W s = ((const W*)a.states)[i];
  const int c = check_invariants_all(L, *P, s);
  if (c < 0) return;
  atomicMin(a.ev, (unsigned long long)make_event(user_check_dkey(L, a, i, s), (c & 1) ? EVK_INV_ERROR : EVK_VIOLATION,
                                                 c >> 1));
}

// ---- Init (compaction.tla:188-202), world == 1: initial state idx goes to
// store position idx, which is also TLC's enumeration order.
template <typename W>
__global__ __launch_bounds__(BLOCK) void k_init_direct(Layout L, u64 n_init, u64* __restrict__ slots, int log2,
                                                       W* __restrict__ states, u64* __restrict__ parents,
                                                       LevelCtr* ctr) {
  const u64 idx = (u64)blockIdx.x * BLOCK + threadIdx.x;
  if (idx >= n_init) return;
  const W s = init_state<W>(L, idx);
  u64 slot;
  const int r = fpset_put(slots, log2, s, mixw(s), &slot);
  if (r < 0) atomicOr(&ctr->overflow, ovf_of(r));
  if (r == 0) atomicOr(&ctr->overflow, (unsigned)OVF_DUP_INIT);
  states[idx] = s;
  parents[idx] = NO_PARENT;
  const int c = check_invariants(L, s);
  if (c >= 0) atomicMin(&ctr->event, make_event(idx, (c & 1) ? EVK_INV_ERROR : EVK_VIOLATION, c >> 1));
}

// ---- Init, world > 1: keep only the initial states this rank owns.
template <typename W>
__global__ __launch_bounds__(BLOCK) void k_init_part(Layout L, u64 n_init, int rank, int world, u64 owner_mask,
                                                     u64* __restrict__ slots, int log2, W* __restrict__ states,
                                                     u64* __restrict__ parents, u64 cap, LevelCtr* ctr) {
  __shared__ W s_st[BLOCK];
  __shared__ u64 s_par[BLOCK];
  __shared__ unsigned s_cnt;
  __shared__ unsigned long long s_base;
  if (threadIdx.x == 0) s_cnt = 0;
  __syncthreads();
  const u64 idx = (u64)blockIdx.x * BLOCK + threadIdx.x;
  bool mine = false;
  W s = 0;
  if (idx < n_init) {
    s = init_state<W>(L, idx);
    if (owner_of(s, owner_mask, world) == rank) {
      u64 slot;
      const int r = fpset_put(slots, log2, s, mixw(s), &slot);
      if (r < 0) atomicOr(&ctr->overflow, ovf_of(r));
      mine = r == 1;
      if (mine) {
        const int c = check_invariants(L, s);
        if (c >= 0) atomicMin(&ctr->event, make_event(idx, (c & 1) ? EVK_INV_ERROR : EVK_VIOLATION, c >> 1));
      }
    }
  }
  stage_append<false, W>(mine, s, NO_PARENT, 0, s_st, s_par, nullptr, &s_cnt);
  __syncthreads();
  if (threadIdx.x == 0) s_base = s_cnt ? atomicAdd(&ctr->n_new, (unsigned long long)s_cnt) : 0;
  __syncthreads();
  const unsigned n = s_cnt;
  const u64 b = s_base;
  if (b + n > cap) {
    if (threadIdx.x == 0) atomicOr(&ctr->overflow, (unsigned)OVF_STORE);
    return;
  }
  for (unsigned i = threadIdx.x; i < n; i += BLOCK) {
    states[b + i] = s_st[i];
    parents[b + i] = s_par[i];
  }
}

// ---- one BFS level ----
template <typename W, bool PRODUCER, bool TLC, bool PART>
__global__ __launch_bounds__(BLOCK) void k_expand(ExpandArgs a) {
  __shared__ W s_st[STAGE_CAP];
  __shared__ u64 s_par[STAGE_CAP];
  __shared__ u64 s_slot[TLC ? STAGE_CAP : 1];
  // PART: the stage also holds the records for other ranks; s_dst = the owner
  // of each staged state (this rank for a new local state)
  __shared__ uint8_t s_dst[PART ? STAGE_CAP : 1];
  __shared__ unsigned s_dn[PART ? 64 : 1], s_dcur[PART ? 64 : 1];
  __shared__ unsigned long long s_db[PART ? 64 : 1];
  __shared__ unsigned s_cnt;
  __shared__ unsigned long long s_base;
  const Layout& L = a.L;
  if (threadIdx.x == 0) s_cnt = 0;
  __syncthreads();

  u64 gen = 0;
  unsigned long long ev = NO_EVENT;

  // emit one successor (all lanes of the wave call this)
  auto emit = [&](bool pred, W t, u64 dkey) {
    bool isnew = false;
    u64 slot = 0;
    bool local = pred;
    if (PART) {
      // a successor owned elsewhere is staged with its owner and leaves for
      // that rank's outbox at the block's flush, which claims room with one
      // atomic per destination per block (per-wave claims on the world's few
      // n_out words serialized at the memory side)
      const int dst = pred ? owner_of(t, a.owner_mask, a.world) : a.rank;
      const bool remote = pred && dst != a.rank;
      local = pred && !remote;
      if (local) {
        const int r = fpset_put(a.slots, a.log2, t, mixw(t), &slot);
        if (r < 0) atomicOr(&a.ctr->overflow, ovf_of(r));
        isnew = r == 1;
        if (isnew) {
          const int c = check_invariants(L, t);
          if (c >= 0) ev = min(ev, (unsigned long long)make_event(dkey, (c & 1) ? EVK_INV_ERROR : EVK_VIOLATION, c >> 1));
        }
      }
      const bool put = remote || isnew;
      const u64 m = __ballot(put);
      if (m) {
        const int leader = __ffsll((long long)m) - 1;
        unsigned base = 0;
        if (__lane_id() == leader) base = atomicAdd(&s_cnt, (unsigned)__popcll(m));
        base = __shfl(base, leader);
        if (put) {
          const unsigned pos = base + (unsigned)__popcll(m & lanemask_lt());
          s_st[pos] = t;
          s_par[pos] = a.rank_tag | dkey;
          s_dst[pos] = (uint8_t)dst;
        }
      }
      return;
    }
    if (local) {
      const int r = fpset_put(a.slots, a.log2, t, mixw(t), &slot);
      if (r < 0) atomicOr(&a.ctr->overflow, ovf_of(r));
      isnew = r == 1;
      if (TLC && r >= 0) atomicMin((unsigned long long*)&a.dkey_slot[slot], (unsigned long long)dkey);
      if (!TLC && isnew) {
        const int c = check_invariants(L, t);
        if (c >= 0) ev = min(ev, (unsigned long long)make_event(dkey, (c & 1) ? EVK_INV_ERROR : EVK_VIOLATION, c >> 1));
      }
    }
    stage_append<TLC, W>(isnew, t, a.rank_tag | dkey, slot, s_st, s_par, s_slot, &s_cnt);
  };

  auto flush = [&]() {
    __syncthreads();
    if (PART) {
      // counting sort of the stage by owner: one n_new / n_out claim per
      // destination, then every state to the store or its rank's outbox
      const unsigned n = s_cnt;
      if (threadIdx.x < (unsigned)a.world) s_dn[threadIdx.x] = s_dcur[threadIdx.x] = 0;
      __syncthreads();
      for (unsigned i = threadIdx.x; i < n; i += BLOCK) atomicAdd(&s_dn[s_dst[i]], 1u);
      __syncthreads();
      if (threadIdx.x < (unsigned)a.world) {
        const unsigned c = s_dn[threadIdx.x];
        unsigned long long* ctr = (int)threadIdx.x == a.rank ? &a.ctr->n_new : &a.ctr->n_out[threadIdx.x];
        s_db[threadIdx.x] = c ? atomicAdd(ctr, (unsigned long long)c) : 0;
      }
      __syncthreads();
      for (unsigned i = threadIdx.x; i < n; i += BLOCK) {
        const int d = s_dst[i];
        const u64 pos = s_db[d] + atomicAdd(&s_dcur[d], 1u);
        if (d == a.rank) {
          if (pos < a.cap_out) {
            reinterpret_cast<W*>(a.states_out)[pos] = s_st[i];
            a.parents_out[pos] = s_par[i];
          } else {
            atomicOr(&a.ctr->overflow, (unsigned)OVF_STORE);
          }
        } else if (pos < a.outbox_cap) {
          u64* rec = a.outbox + 2 * ((u64)d * a.outbox_cap + pos);
          rec[0] = (u64)s_st[i];  // PART: one-word states only (tlcg_create)
          rec[1] = s_par[i];
        } else {
          atomicOr(&a.ctr->overflow, (unsigned)OVF_OUTBOX);
        }
      }
      __syncthreads();
      if (threadIdx.x == 0) s_cnt = 0;
      __syncthreads();
      return;
    }
    if (threadIdx.x == 0) s_base = s_cnt ? atomicAdd(&a.ctr->n_new, (unsigned long long)s_cnt) : 0;
    __syncthreads();
    const unsigned n = s_cnt;
    const u64 b = s_base;
    if (b + n <= a.cap_out) {
      for (unsigned i = threadIdx.x; i < n; i += BLOCK) {
        reinterpret_cast<W*>(a.states_out)[b + i] = s_st[i];
        a.parents_out[b + i] = s_par[i];
        if (TLC) a.slot_out[b + i] = s_slot[i];
      }
    } else if (threadIdx.x == 0 && n) {
      atomicOr(&a.ctr->overflow, (unsigned)OVF_STORE);
    }
    __syncthreads();
    if (threadIdx.x == 0) s_cnt = 0;
    __syncthreads();
  };

  // room check at a block-uniform point: flush if `upcoming` more emits could overflow the stage
  auto reserve = [&](int upcoming) {
    __syncthreads();
    const unsigned n = s_cnt;
    __syncthreads();
    if (n + (unsigned)upcoming * BLOCK > (unsigned)STAGE_CAP) flush();
  };

  constexpr int kItems = PRODUCER ? 1 : ITEMS;
  const u64 per_chunk = (u64)BLOCK * kItems;
  const u64 ord_last = (1ull << L.ord_bits) - 1;
  for (u64 c0 = (u64)blockIdx.x * per_chunk; c0 < a.n_front; c0 += (u64)gridDim.x * per_chunk) {
#pragma unroll 1
    for (int it = 0; it < kItems; ++it) {
      const u64 pi = c0 + (u64)it * BLOCK + threadIdx.x;
      const bool valid = pi < a.n_front;
      const W s = valid ? reinterpret_cast<const W*>(a.frontier)[pi] : (W)0;
      const u64 dk0 = (a.front_gidx0 + pi) << L.ord_bits;
      int nsucc = 0;
      if (PRODUCER) {  // Producer, compaction.tla:83-87
        const int len = st_len(L, s);
        const bool can = valid && len < L.N;
#pragma unroll 1
        for (int j = 0; j < L.nkv; ++j) {
          if ((j & 3) == 0) reserve(6);
          emit(can, can ? producer_succ(L, s, len, j) : (W)0, dk0 | (u64)j);
        }
        nsucc += can ? L.nkv : 0;
        reserve(2);
      }
      // the compactor disjuncts, compaction.tla:221-226
      W t = 0;
      int act = 0;
      const int r = valid ? compactor_step(L, s, &t, &act) : 0;
      if (r == 2) ev = min(ev, (unsigned long long)make_event(dk0 | (u64)ordinal_of(L, act, 0), EVK_ACTION_ERROR, act));
      nsucc += (r == 1);
      emit(r == 1, t, dk0 | (u64)ordinal_of(L, act, 0));
      // BrokerCrash, compaction.tla:227
      W t2 = 0;
      const bool en2 = valid && crash_step(L, s, &t2);
      nsucc += en2;
      emit(en2, t2, dk0 | (u64)ordinal_of(L, ACT_CRASH, 0));
      // Consumer / Terminating: stuttering successors, generated but never new
      if (valid) nsucc += selfloop_count(L, s);
      gen += (u64)nsucc;
      if (valid && nsucc == 0 && L.check_deadlock)
        ev = min(ev, (unsigned long long)make_event(dk0 | ord_last, EVK_DEADLOCK, 0));
    }
    flush();
  }
  gen = wave_sum_u64(gen);
  if (__lane_id() == 0 && gen) atomicAdd(&a.ctr->generated, (unsigned long long)gen);
  if (ev != NO_EVENT) atomicMin(&a.ctr->event, ev);
}


// ---- the fast path of one BFS level (no Producer, discovery order not kept,
// successors stay on this rank): every thread takes IT parents, derives all
// their candidate successors first, then issues the FPSet probes of all of
// them together (2*IT independent loads / CASes in flight per lane) before
// staging the new ones.  PROBE 0: load, CAS only on an empty slot; PROBE 1:
// CAS straight away (one round trip, an atomic on every probe).
template <int IT, int PROBE>
__global__ __launch_bounds__(BLOCK) void k_expand_fast(ExpandArgs a) {
  constexpr int NC = 2 * IT;
  constexpr int CAP = BLOCK * NC;
  __shared__ u64 s_st[CAP];
  __shared__ u64 s_par[CAP];
  __shared__ unsigned s_cnt;
  __shared__ unsigned long long s_base;
  const Layout& L = a.L;
  if (threadIdx.x == 0) s_cnt = 0;
  __syncthreads();
  u64 gen = 0;
  unsigned long long ev = NO_EVENT;
  const u64 per_chunk = (u64)BLOCK * IT;
  const u64 ord_last = (1ull << L.ord_bits) - 1;
  const int sh = 64 - a.log2;
  const u64 mask = (1ull << a.log2) - 1;
  const int ord_crash = ordinal_of(L, ACT_CRASH, 0);
  for (u64 c0 = (u64)blockIdx.x * per_chunk; c0 < a.n_front; c0 += (u64)gridDim.x * per_chunk) {
    u64 s[IT];
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const u64 pi = c0 + (u64)it * BLOCK + threadIdx.x;
      s[it] = pi < a.n_front ? a.frontier[pi] : 0;
    }
    u64 cand[NC], dk[NC], pos[NC], v[NC];
    bool has[NC];
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const u64 pi = c0 + (u64)it * BLOCK + threadIdx.x;
      const bool valid = pi < a.n_front;
      const u64 dk0 = (a.front_gidx0 + pi) << L.ord_bits;
      u64 t = 0;
      int act = 0;
      const int r = valid ? compactor_step(L, s[it], &t, &act) : 0;
      if (r == 2) ev = min(ev, (unsigned long long)make_event(dk0 | (u64)ordinal_of(L, act, 0), EVK_ACTION_ERROR, act));
      cand[2 * it] = t;
      has[2 * it] = r == 1;
      dk[2 * it] = dk0 | (u64)ordinal_of(L, act, 0);
      u64 t2 = 0;
      has[2 * it + 1] = valid && crash_step(L, s[it], &t2);
      cand[2 * it + 1] = t2;
      dk[2 * it + 1] = dk0 | (u64)ord_crash;
      int nsucc = (int)has[2 * it] + (int)has[2 * it + 1] + (valid ? selfloop_count(L, s[it]) : 0);
      gen += (u64)nsucc;
      if (valid && nsucc == 0 && L.check_deadlock)
        ev = min(ev, (unsigned long long)make_event(dk0 | ord_last, EVK_DEADLOCK, 0));
    }
    // first probe of every candidate, all in flight together
#pragma unroll
    for (int c = 0; c < NC; ++c) pos[c] = mix64(cand[c]) >> sh;
    // after this, v[c] == 0 means "inserted by this lane" (CAS returned 0);
    // v[c] == key means present; anything else: the slot holds another state
    if (PROBE == 0) {
#pragma unroll
      for (int c = 0; c < NC; ++c) v[c] = has[c] ? __builtin_nontemporal_load(&a.slots[pos[c]]) : 1;
#pragma unroll
      for (int c = 0; c < NC; ++c)
        if (has[c] && v[c] == 0)
          v[c] = atomicCAS((unsigned long long*)&a.slots[pos[c]], 0ull, (unsigned long long)(cand[c] | SLOT_TAG));
    } else {
#pragma unroll
      for (int c = 0; c < NC; ++c)
        v[c] = has[c] ? atomicCAS((unsigned long long*)&a.slots[pos[c]], 0ull, (unsigned long long)(cand[c] | SLOT_TAG))
                      : 1;
    }
    // resolve: new / seen; probe on past slots held by other states
    bool isnew[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      isnew[c] = false;
      if (!has[c]) continue;
      const u64 key = cand[c] | SLOT_TAG;
      if (v[c] == 0) { isnew[c] = true; continue; }
      if (v[c] == key) continue;
      u64 slot;
      const int r = fpset_put_from(a.slots, mask, key, (pos[c] + 1) & mask, &slot);
      if (r < 0) atomicOr(&a.ctr->overflow, (unsigned)OVF_FPSET);
      isnew[c] = r == 1;
    }
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      if (isnew[c]) {
        const int q = check_invariants(L, cand[c]);
        if (q >= 0) ev = min(ev, (unsigned long long)make_event(dk[c], (q & 1) ? EVK_INV_ERROR : EVK_VIOLATION, q >> 1));
      }
      stage_append<false, u64>(isnew[c], cand[c], a.rank_tag | dk[c], 0, s_st, s_par, nullptr, &s_cnt);
    }
    // flush the stage: one global atomic per block chunk
    __syncthreads();
    if (threadIdx.x == 0) s_base = s_cnt ? atomicAdd(&a.ctr->n_new, (unsigned long long)s_cnt) : 0;
    __syncthreads();
    const unsigned n = s_cnt;
    const u64 b = s_base;
    if (b + n <= a.cap_out) {
      for (unsigned i = threadIdx.x; i < n; i += BLOCK) {
        a.states_out[b + i] = s_st[i];
        a.parents_out[b + i] = s_par[i];
      }
    } else if (threadIdx.x == 0 && n) {
      atomicOr(&a.ctr->overflow, (unsigned)OVF_STORE);
    }
    __syncthreads();
    if (threadIdx.x == 0) s_cnt = 0;
    __syncthreads();
  }
  gen = wave_sum_u64(gen);
  if (__lane_id() == 0 && gen) atomicAdd(&a.ctr->generated, (unsigned long long)gen);
  if (ev != NO_EVENT) atomicMin(&a.ctr->event, ev);
}

// ---- the fast path of a Producer level (discovery order not kept, local
// partition, one-word states): a thread takes two parents; their successors
// are probed in chunks whose FPSet probes are all in flight together (a load
// each, then a CAS on the empty slots), so a thread waits on a chunk of
// scattered round trips at once instead of one per successor, and the
// block's LDS stage is flushed once per chunk.  Producer's |KeySet| x
// |ValueSet| successors (compaction.tla:83-87) come in chunks of PB, and a
// block none of whose parents can produce (Len(messages) = N: most states)
// skips them; the compactor and BrokerCrash successors of both parents form
// one last chunk of four.
template <int PB>
__global__ __launch_bounds__(BLOCK) void k_expand_prod(ExpandArgs a) {
  constexpr int CW = PB > 4 ? PB : 4;  // widest chunk
  constexpr int CAP = BLOCK * CW;
  __shared__ u64 s_st[CAP];
  __shared__ u64 s_par[CAP];
  __shared__ unsigned s_cnt;
  __shared__ unsigned long long s_base;
  const Layout& L = a.L;
  if (threadIdx.x == 0) s_cnt = 0;
  __syncthreads();
  u64 gen = 0;
  unsigned long long ev = NO_EVENT;
  const u64 ord_last = (1ull << L.ord_bits) - 1;
  const int sh = 64 - a.log2;
  const u64 mask = (1ull << a.log2) - 1;
  const int ord_crash = ordinal_of(L, ACT_CRASH, 0);
  // probe, insert, check and stage NC candidates, then flush the stage
  auto chunk = [&](auto ncw, const u64* cand, const bool* has, const u64* dk) {
    constexpr int NC = decltype(ncw)::value;
    u64 pos[NC], v[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) pos[c] = mix64(cand[c]) >> sh;
#pragma unroll
    for (int c = 0; c < NC; ++c) v[c] = has[c] ? __builtin_nontemporal_load(&a.slots[pos[c]]) : 1;
#pragma unroll
    for (int c = 0; c < NC; ++c)
      if (has[c] && v[c] == 0)
        v[c] = atomicCAS((unsigned long long*)&a.slots[pos[c]], 0ull, (unsigned long long)(cand[c] | SLOT_TAG));
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      bool isnew = false;
      if (has[c]) {
        const u64 key = cand[c] | SLOT_TAG;
        if (v[c] == 0) {
          isnew = true;
        } else if (v[c] != key) {  // the first slot holds another state: probe on
          u64 slot;
          const int rr = fpset_put_from(a.slots, mask, key, (pos[c] + 1) & mask, &slot);
          if (rr < 0) atomicOr(&a.ctr->overflow, (unsigned)OVF_FPSET);
          isnew = rr == 1;
        }
        if (isnew) {
          const int q = check_invariants(L, cand[c]);
          if (q >= 0) ev = min(ev, (unsigned long long)make_event(dk[c], (q & 1) ? EVK_INV_ERROR : EVK_VIOLATION, q >> 1));
        }
      }
      stage_append<false, u64>(isnew, cand[c], a.rank_tag | dk[c], 0, s_st, s_par, nullptr, &s_cnt);
    }
    __syncthreads();
    if (threadIdx.x == 0) s_base = s_cnt ? atomicAdd(&a.ctr->n_new, (unsigned long long)s_cnt) : 0;
    __syncthreads();
    const unsigned n = s_cnt;
    const u64 b = s_base;
    if (b + n <= a.cap_out) {
      for (unsigned i = threadIdx.x; i < n; i += BLOCK) {
        a.states_out[b + i] = s_st[i];
        a.parents_out[b + i] = s_par[i];
      }
    } else if (threadIdx.x == 0 && n) {
      atomicOr(&a.ctr->overflow, (unsigned)OVF_STORE);
    }
    __syncthreads();
    if (threadIdx.x == 0) s_cnt = 0;
    __syncthreads();
  };
  using I4 = std::integral_constant<int, 4>;
  using IPB = std::integral_constant<int, PB>;
  for (u64 c0 = (u64)blockIdx.x * BLOCK * 2; c0 < a.n_front; c0 += (u64)gridDim.x * BLOCK * 2) {
    u64 s[2], dk0[2], t[2], t2[2];
    int len[2], act[2];
    bool can[2], en1[2], en2[2];
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const u64 pi = c0 + (u64)it * BLOCK + threadIdx.x;
      const bool valid = pi < a.n_front;
      s[it] = valid ? a.frontier[pi] : 0;
      dk0[it] = (a.front_gidx0 + pi) << L.ord_bits;
      len[it] = st_len(L, s[it]);
      can[it] = valid && len[it] < L.N;  // Producer's guard, :84
      t[it] = 0;
      act[it] = 0;
      const int r = valid ? compactor_step(L, s[it], &t[it], &act[it]) : 0;
      if (r == 2)
        ev = min(ev, (unsigned long long)make_event(dk0[it] | (u64)ordinal_of(L, act[it], 0), EVK_ACTION_ERROR, act[it]));
      en1[it] = r == 1;
      t2[it] = 0;
      en2[it] = valid && crash_step(L, s[it], &t2[it]);
      const int nsucc = (can[it] ? L.nkv : 0) + (int)en1[it] + (int)en2[it] + (valid ? selfloop_count(L, s[it]) : 0);
      gen += (u64)nsucc;
      if (valid && nsucc == 0 && L.check_deadlock)
        ev = min(ev, (unsigned long long)make_event(dk0[it] | ord_last, EVK_DEADLOCK, 0));
    }
    if (__syncthreads_or(can[0] || can[1])) {  // block-uniform
#pragma unroll 1
      for (int it = 0; it < 2; ++it)
#pragma unroll 1
        for (int j0 = 0; j0 < L.nkv; j0 += PB) {
          u64 cand[PB], dk[PB];
          bool has[PB];
#pragma unroll
          for (int c = 0; c < PB; ++c) {
            const int j = j0 + c;
            has[c] = can[it] && j < L.nkv;
            cand[c] = has[c] ? producer_succ(L, s[it], len[it], j) : 0;
            dk[c] = dk0[it] | (u64)j;
          }
          chunk(IPB(), cand, has, dk);
        }
    }
    const u64 cand[4] = {t[0], t2[0], t[1], t2[1]};
    const bool has[4] = {en1[0], en2[0], en1[1], en2[1]};
    const u64 dk[4] = {dk0[0] | (u64)ordinal_of(L, act[0], 0), dk0[0] | (u64)ord_crash,
                       dk0[1] | (u64)ordinal_of(L, act[1], 0), dk0[1] | (u64)ord_crash};
    chunk(I4(), cand, has, dk);
  }
  gen = wave_sum_u64(gen);
  if (__lane_id() == 0 && gen) atomicAdd(&a.ctr->generated, (unsigned long long)gen);
  if (ev != NO_EVENT) atomicMin(&a.ctr->event, ev);
}

// ---- TLC order: gather each new state's minimal discovery key
__global__ __launch_bounds__(BLOCK) void k_gather_dkey(u64 n, const u64* __restrict__ slot_new,
                                                       const u64* __restrict__ dkey_slot, u64* __restrict__ dk) {
  const u64 i = (u64)blockIdx.x * BLOCK + threadIdx.x;
  if (i < n) dk[i] = dkey_slot[slot_new[i]];
}

// ---- TLC order: write the level back in discovery order, parent = first
// discoverer, invariants on each new state keyed by its discovery key.
template <typename W>
__global__ __launch_bounds__(BLOCK) void k_tlc_finish(Layout L, u64 n, const W* __restrict__ st_sorted,
                                                      const u64* __restrict__ dk_sorted, W* __restrict__ states,
                                                      u64* __restrict__ parents, u64 rank_tag, LevelCtr* ctr) {
  const u64 i = (u64)blockIdx.x * BLOCK + threadIdx.x;
  if (i >= n) return;
  const W s = st_sorted[i];
  const u64 dk = dk_sorted[i];
  states[i] = s;
  parents[i] = rank_tag | dk;
  const int c = check_invariants(L, s);
  if (c >= 0) atomicMin(&ctr->event, make_event(dk, (c & 1) ? EVK_INV_ERROR : EVK_VIOLATION, c >> 1));
}

// ---- FPSet growth: re-insert every stored state
template <typename W>
__global__ __launch_bounds__(BLOCK) void k_reinsert(const W* __restrict__ states, u64 n, u64* __restrict__ slots,
                                                    int log2, LevelCtr* ctr) {
  const u64 i = (u64)blockIdx.x * BLOCK + threadIdx.x;
  if (i >= n) return;
  const W s = states[i];
  u64 slot;
  const int r = fpset_put(slots, log2, s, mixw(s), &slot);
  if (r < 0) atomicOr(&ctr->overflow, ovf_of(r));
}

// ---- host FPSet tier (opts.fpset_spill).  The host runs hold the mixed keys
// mix64(state) (a bijection, so exact) in sorted order; HBM holds a blocked
// Bloom filter over them: 2^log2b blocks of 64 bytes, 6 bits per key.
__device__ __forceinline__ u64 bloom_hash(u64 key) { return mix64(key ^ 0x5851F42D4C957F2Dull); }

__global__ __launch_bounds__(BLOCK) void k_bloom_insert(const u64* __restrict__ keys, u64 n, u64* __restrict__ bloom,
                                                        int log2b) {
  const u64 i = (u64)blockIdx.x * BLOCK + threadIdx.x;
  if (i >= n) return;
  const u64 h = bloom_hash(keys[i]);
  u64* b = bloom + 8 * (h >> (64 - log2b));
  const u64 h2 = mix64(h);
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    const unsigned bit = (unsigned)(h2 >> (9 * j)) & 511u;
    atomicOr((unsigned long long*)&b[bit >> 6], 1ull << (bit & 63));
  }
}

// the level's new states [0, n) (new to the HBM table): queue the ones the
// filter cannot rule out of the host runs as {mixed key, position}
__global__ __launch_bounds__(BLOCK) void k_tier_filter(const u64* __restrict__ states, u64 n,
                                                       const u64* __restrict__ bloom, int log2b, u64* __restrict__ q_key,
                                                       u64* __restrict__ q_pos, unsigned long long* q_n) {
  const u64 i = (u64)blockIdx.x * BLOCK + threadIdx.x;
  bool maybe = false;
  u64 key = 0;
  if (i < n) {
    key = mix64(states[i]);
    const u64 h = bloom_hash(key);
    const u64* b = bloom + 8 * (h >> (64 - log2b));
    const u64 h2 = mix64(h);
    maybe = true;
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      const unsigned bit = (unsigned)(h2 >> (9 * j)) & 511u;
      maybe = maybe && ((b[bit >> 6] >> (bit & 63)) & 1);
    }
  }
  const u64 m = __ballot(maybe);
  if (!m) return;
  unsigned long long base = 0;
  if (__lane_id() == __ffsll((unsigned long long)m) - 1) base = atomicAdd(q_n, (unsigned long long)__popcll(m));
  base = __shfl(base, __ffsll((unsigned long long)m) - 1);
  if (maybe) {
    const u64 p = base + __popcll(m & lanemask_lt());
    q_key[p] = key;
    q_pos[p] = i;
  }
}

// keep[pos] = 0 for the queued states the host runs hold
__global__ __launch_bounds__(BLOCK) void k_tier_mark(const u64* __restrict__ q_pos, const unsigned char* __restrict__ dup,
                                                     u64 m, unsigned char* __restrict__ keep) {
  const u64 j = (u64)blockIdx.x * BLOCK + threadIdx.x;
  if (j < m && dup[j]) keep[q_pos[j]] = 0;
}

__global__ __launch_bounds__(BLOCK) void k_mix_keys(const u64* __restrict__ states, u64 n, u64* __restrict__ keys) {
  const u64 i = (u64)blockIdx.x * BLOCK + threadIdx.x;
  if (i < n) keys[i] = mix64(states[i]);
}

// ---- world > 1: insert successors received from other ranks.  Each thread
// takes ABSORB_IT records and issues their first FPSet probes together (a
// load each, then a CAS on the empty slots), as k_expand_fast does, so
// ABSORB_IT scattered round trips are in flight per lane instead of one.
constexpr int ABSORB_IT = 4;
__global__ __launch_bounds__(BLOCK) void k_absorb(Layout L, const u64* __restrict__ recs, u64 n,
                                                  u64* __restrict__ slots, int log2, u64* __restrict__ states_out,
                                                  u64* __restrict__ parents_out, u64 cap, LevelCtr* ctr) {
  __shared__ u64 s_st[BLOCK * ABSORB_IT], s_par[BLOCK * ABSORB_IT];
  __shared__ unsigned s_cnt;
  __shared__ unsigned long long s_base;
  if (threadIdx.x == 0) s_cnt = 0;
  __syncthreads();
  const u64 mask = (1ull << log2) - 1;
  const u64 i0 = (u64)blockIdx.x * BLOCK * ABSORB_IT + threadIdx.x;
  u64 t[ABSORB_IT], ref[ABSORB_IT], pos[ABSORB_IT], v[ABSORB_IT];
  bool has[ABSORB_IT];
#pragma unroll
  for (int k = 0; k < ABSORB_IT; ++k) {
    const u64 i = i0 + (u64)k * BLOCK;
    has[k] = i < n;
    t[k] = has[k] ? recs[2 * i] : 0;
    ref[k] = has[k] ? recs[2 * i + 1] : 0;
    pos[k] = mix64(t[k]) >> (64 - log2);
  }
#pragma unroll
  for (int k = 0; k < ABSORB_IT; ++k) v[k] = has[k] ? __builtin_nontemporal_load(&slots[pos[k]]) : 1;
#pragma unroll
  for (int k = 0; k < ABSORB_IT; ++k)
    if (has[k] && v[k] == 0) v[k] = atomicCAS((unsigned long long*)&slots[pos[k]], 0ull, (unsigned long long)(t[k] | SLOT_TAG));
#pragma unroll
  for (int k = 0; k < ABSORB_IT; ++k) {
    bool isnew = false;
    if (has[k]) {
      const u64 key = t[k] | SLOT_TAG;
      if (v[k] == 0) {
        isnew = true;
      } else if (v[k] != key) {  // the first slot holds another state: probe on
        u64 slot;
        const int r = fpset_put_from(slots, mask, key, (pos[k] + 1) & mask, &slot);
        if (r < 0) atomicOr(&ctr->overflow, (unsigned)OVF_FPSET);
        isnew = r == 1;
      }
      if (isnew) {
        const int c = check_invariants(L, t[k]);
        // keyed by inbox position, tagged with bit 51 (resolved on the host)
        if (c >= 0)
          atomicMin(&ctr->event, make_event((1ull << 51) | (i0 + (u64)k * BLOCK), (c & 1) ? EVK_INV_ERROR : EVK_VIOLATION,
                                            c >> 1));
      }
    }
    stage_append<false, u64>(isnew, t[k], ref[k], 0, s_st, s_par, nullptr, &s_cnt);
  }
  __syncthreads();
  if (threadIdx.x == 0) s_base = s_cnt ? atomicAdd(&ctr->n_new, (unsigned long long)s_cnt) : 0;
  __syncthreads();
  const unsigned m = s_cnt;
  const u64 b = s_base;
  if (b + m > cap) {
    if (threadIdx.x == 0) atomicOr(&ctr->overflow, (unsigned)OVF_STORE);
    return;
  }
  for (unsigned k = threadIdx.x; k < m; k += BLOCK) {
    states_out[b + k] = s_st[k];
    parents_out[b + k] = s_par[k];
  }
}

// TLC order: the new level is sorted by first-discovery key, so the states a
// parent discovered first form one run of equal parent_gidx.  hist[len] +=
// 1 for every run (len <= OUTDEG_BINS - 1: nkv + 2 new states per parent).
constexpr int OUTDEG_BINS = 4100;
__global__ __launch_bounds__(BLOCK) void k_child_runs(const u64* __restrict__ parents, u64 n, int ord_bits,
                                                      unsigned long long* __restrict__ hist) {
  const u64 i = (u64)blockIdx.x * BLOCK + threadIdx.x;
  if (i >= n) return;
  const u64 km = (1ull << 56) - 1;
  const u64 p = (parents[i] & km) >> ord_bits;
  if (i > 0 && ((parents[i - 1] & km) >> ord_bits) == p) return;  // not the start of a run
  u64 len = 1;
  while (i + len < n && ((parents[i + len] & km) >> ord_bits) == p) ++len;
  atomicAdd(&hist[len < (u64)OUTDEG_BINS ? len : (u64)OUTDEG_BINS - 1], 1ull);
}

inline unsigned grid_for(u64 n, u64 per_block, unsigned cap) {
  u64 g = (n + per_block - 1) / per_block;
  if (g < 1) g = 1;
  return (unsigned)std::min<u64>(g, cap);
}

}  // namespace

// ======================= host runtime =======================

struct tlcg_ctx {
  tlcg_model model;
  tlcg_opts opts;
  HostModel hm;
  std::string user_defs;                 // model.user_defs points here (tlcg_create copies the caller's text)
  std::string user_src;                  // the user invariants as device code (user_device_source), for jit_build
  uint32_t comp_mult = 0, tree_mult = 0;  // tuned slot-hash multipliers (0: not yet)
  uint32_t tree_disp_mult = 0;               // the tree's closed-mode slot displacements (build_slot_disp)
  uint16_t tree_disp[TREE_DISP] = {};
  bool no_tree = false;                   // the ranks fell back from the sharded component tree (run_ranks)
  bool tree_event = false;                // the last tree run raised an error (Producer modelled: TLC order reports it)
  bool tlc_switched = false;              // this run took TLC order for a tree error (opts.tlc_order restored at tlcg_init)
  u64 range_hi = 0;                       // closed, one rank: run only initial states [0, range_hi) (TLC stop statistics)
  u64 ev_comp = ~0ull;                    // closed partitions, on-chip engines: the initial state of the error's component
  // a run whose level 0 is one given state instead of Init (the Producer
  // tree's error report: a TLC-order run over one subtree, producer_error)
  bool seed_valid = false;
  u128 seed_state = 0;
  // TLC's stop statistics worked out with the run (the Producer tree's error report)
  bool stop_cached = false;
  u64 stop_g = 0, stop_d = 0, stop_q = 0;
  // the component tree's layout (Producer modelled, one rank): per layer, the
  // global index of its first chunk and of its first component
  std::vector<u64> tree_layer_gbase, tree_layer_cbase;
  bool tree_codes = false;                // the store holds the tree's closed-mode component codes (tree_body.h)
  u64 tree_r0 = 0;                        //   of the components of initial states tree_r0, tree_r0 + 1, ..
  UserProg* d_prog = nullptr;            // the user invariants' program on the device (user_inv.h)
  unsigned long long* d_uev = nullptr;   // k_user_check's event (min)
  int words = 1;  // u64 words per state: 1, or 2 for wide layouts (> 63 bits)
  int device = 0;
  hipStream_t stream = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr, e2 = nullptr;
  // FPSet
  u64* d_slots = nullptr;
  int log2 = 0;
  u64* d_dkey_slot = nullptr;  // TLC order
  // state store (all levels) + parent log
  u64* d_states = nullptr;
  u64* d_parents = nullptr;
  u64 cap = 0;  // device slots; they hold the states with gidx in [win, win + cap)
  // host spill (opts.spill): committed states below `win` live in pinned host
  // chunks, each a gidx range [g0, g0 + n) of states and parent refs
  struct HostChunk {
    u64 g0, n;
    u64* st;
    u64* par;
  };
  std::vector<HostChunk> hchunks;
  u64 win = 0;
  // registered host blocks not in use (kept for the next run; freed by tlcg_destroy)
  struct HostBlock {
    void* p;
    size_t bytes;
  };
  std::vector<HostBlock> host_pool;
  std::vector<std::pair<void*, size_t>> host_sizes;  // every registered block
  // host FPSet tier (opts.fpset_spill): the states [0, t0_base) are held by
  // sorted runs of mixed keys in host memory (one per flush) and summarized by
  // an HBM Bloom filter; the HBM table holds the states from t0_base on
  struct Run {
    u64* keys;
    u64 n;
  };
  std::vector<Run> runs;
  u64 t0_base = 0;
  u64* d_bloom = nullptr;
  int bloom_log2 = 0;  // 2^bloom_log2 blocks of 64 bytes
  // level filter scratch (grown on demand)
  u64* d_q = nullptr;  // [2][cap]: queued keys, positions (then sorted copies)
  unsigned char* d_keep = nullptr;
  u64* d_sel = nullptr;  // selected states / parents
  void* d_ftmp = nullptr;
  size_t ftmp_bytes = 0;
  u64 filt_cap = 0;
  unsigned long long* d_qn = nullptr;
  u64 tier_queued = 0, tier_dups = 0;  // filter "maybe"s, and the ones the host runs held
  double tier_ms[4] = {0, 0, 0, 0};     // flush, Bloom filter pass, host lookups, compaction (wall)
  // TLC-order scratch
  u64* d_slot_new = nullptr;
  u64* d_dk = nullptr;
  u64* d_dk2 = nullptr;
  u64* d_st2 = nullptr;
  void* d_sort_tmp = nullptr;
  size_t sort_tmp_bytes = 0;
  u64 scratch_cap = 0;
  // partition exchange
  u64* d_outbox = nullptr;
  u64 outbox_cap = 0;  // records per destination
  u64* d_inbox = nullptr;
  u64 inbox_cap = 0;
  // engine of the current run (TLCG_ENGINE_GLOBAL or _COMPONENT)
  int engine = TLCG_ENGINE_GLOBAL;
  // component engine: results, scratch, and where each pass put its components
  struct CompPass {
    int K;
    u64 store_base, r0, n;
    std::vector<u64> list;  // initial-state indices (cascade passes); empty: range [r0, r0 + n)
    bool codes = false;     // the store holds 32-bit records (comp_record), not words + parents
  };
  std::vector<CompPass> passes;
  std::vector<u64> comp_levels;
  std::vector<u64> comp_level_gen;  // successors generated by expanding each level
  u64 comp_init = 0;                // initial states of this rank
  u64 comp_generated = 0, comp_distinct = 0, comp_store_used = 0;
  unsigned long long* d_comp = nullptr;  // lvl[COMP_MAXLV], totals[2], event, ovf_n, outdeg[3], lvl_gen[COMP_MAXLV]
  unsigned long long* h_comp = nullptr;
  bool comp_clean = false;  // d_comp holds zeros (and the event's ~0): k_comp_finish reset it
  // the code pass's 32-bit records (comp_record), in their own buffer: global
  // indices [0, slots) of that pass live here, and the state store's device
  // window starts after them (win), so the store holds only the cascade passes
  uint32_t* d_crec = nullptr;
  u64 crec_cap = 0;
  u64* d_ovf[2] = {nullptr, nullptr};
  u64 ovf_cap = 0;
  // layout-specialized kernels (jit.cpp): 0 untried, 1 built, -1 failed (precompiled ones used)
  JitKernels jit;
  tlcg_ctx* sub = nullptr;  // the Producer tree's subtree runs (producer_error), kept for the next error
  u64 sub_cap = 0;          // its state capacity
  JitUserCheck ujit;  // the global engine's user-invariant check as device code
  int ujit_state = 0; // 0 not built, 1 built, 2 borrowed from the context that made this one, -1 failed
                      // (k_user_check interprets)
  int jit_state = 0;
  bool jit_used = false;
  bool comp_code = false;  // the component engine's first pass runs component codes
  // component-tree engine (tree.h): depths and sizes of every component's chunk, counters
  uint8_t* d_tree_dep = nullptr;
  uint32_t* d_tree_n = nullptr;
  u64 tree_slots = 0, tree_comps = 0;  // capacities of the two arrays
  unsigned long long* d_tree_ctr = nullptr;  // lvl[TREE_MAXLV], lvl_gen[TREE_MAXLV], flags
  unsigned long long* h_tree_ctr = nullptr;
  int tree_cap = 0;  // slots per component of the last tree run (0: none)
  std::string jit_error;
  u64 pending = 0;      // states appended to the current level, not yet committed
  // kernel variant (tuning; env TLCG_FAST_ITEMS / TLCG_PROBE / TLCG_GRID)
  int fast_items = 2;   // parents per thread in k_expand_fast (0 = general kernel)
  int probe_mode = 0;   // 0 load-then-CAS, 1 CAS-only
  unsigned grid_cap = 16384;
  bool closed = false;  // partition by immutable `messages`: successors never leave the rank
  // counters
  LevelCtr* d_ctr = nullptr;
  LevelCtr* h_ctr = nullptr;
  LevelCtr* d_aux = nullptr;  // counters of FPSet rebuilds (never the level's)
  LevelCtr* h_aux = nullptr;
  // run state
  std::vector<u64> level_base;  // level_base[d] = gidx of the first state of level d
  std::vector<u64> gen_at;      // gen_at[d] = generated before level d was expanded (TLC stop statistics)
  // TLC's outdegree statistics: outdeg[k] = expanded states that discovered k
  // new states; kept when the parent log is TLC's (TLC order, component engine)
  std::vector<u64> outdeg;
  bool outdeg_valid = false;
  unsigned long long* d_runs = nullptr;  // [OUTDEG_BINS] device histogram of child runs
  u64 generated = 0;
  int status = TLCG_RUNNING;
  u64 ev_word = NO_EVENT;
  int ev_level = -1;  // level whose expansion raised the event (0 = Init)
  u128 ev_state = 0;
  u64 ev_parent_gidx = NO_PARENT;
  u64 ev_parent_ref = NO_PARENT;
  int ev_action = -1;
  // the counterexample of a multi-rank run, walked across the ranks' stores
  // by trace_ranks (every rank holds it); tlcg_trace_words returns it
  bool xtrace_valid = false;
  std::vector<u128> xtrace_states;
  std::vector<int> xtrace_acts;
  double kernel_ms = 0, expand_ms = 0;
  u64 levels_redone = 0;
  u64 owner_mask = ~0ull;
  std::string err;
  bool inited = false;
  void* comm = nullptr;  // RCCL state (exchange.cpp), tlcg_comm_init
};

namespace tlcg {
int ctx_device(const tlcg_ctx* c) { return c->opts.device; }
int ctx_engine(const tlcg_ctx* c) { return c->engine; }
uint64_t ctx_inbox_cap(const tlcg_ctx* c) { return c->inbox_cap; }
void ctx_disable_tree(tlcg_ctx* c) { c->no_tree = true; }
void ctx_rank_world(const tlcg_ctx* c, int* rank, int* world) {
  *rank = c->opts.rank;
  *world = c->opts.world;
}
void*& ctx_comm(tlcg_ctx* c) { return c->comm; }
void ctx_set_error(tlcg_ctx* c, const std::string& e) { c->err = e; }
}  // namespace tlcg

namespace {

#define HIPCHK(expr)                                                              \
  do {                                                                            \
    hipError_t _e = (expr);                                                       \
    if (_e != hipSuccess) {                                                       \
      c->err = std::string(#expr) + ": " + hipGetErrorString(_e);                 \
      return false;                                                               \
    }                                                                             \
  } while (0)
// the same for the int-returning entry points (< 0 = error)
#define HIPCHK_U(expr)                                                            \
  do {                                                                            \
    hipError_t _e = (expr);                                                       \
    if (_e != hipSuccess) {                                                       \
      c->err = std::string(#expr) + ": " + hipGetErrorString(_e);                 \
      return ~0ull;                                                               \
    }                                                                             \
  } while (0)

#define HIPCHK_I(expr)                                                            \
  do {                                                                            \
    hipError_t _e = (expr);                                                       \
    if (_e != hipSuccess) {                                                       \
      c->err = std::string(#expr) + ": " + hipGetErrorString(_e);                 \
      return -10;                                                                 \
    }                                                                             \
  } while (0)

// Every entry point that allocates, copies or launches makes the context's
// device current for its call: contexts of several devices can then be
// driven from any host thread (tlc-hip -gpus N runs one thread per device).
struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(const tlcg_ctx* c);
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

u64 distinct_of(const tlcg_ctx* c) { return c->level_base.empty() ? 0 : c->level_base.back(); }
DeviceGuard::DeviceGuard(const tlcg_ctx* c) {
  int cur = -1;
  if (c && hipGetDevice(&cur) == hipSuccess && cur != c->opts.device && hipSetDevice(c->opts.device) == hipSuccess)
    prev = cur;
}

// device address of the state / parent ref with global index g (g >= win)
u64* dev_state(tlcg_ctx* c, u64 g) { return c->d_states + (g - c->win) * c->words; }
u64* dev_parent(tlcg_ctx* c, u64 g) { return c->d_parents + (g - c->win); }
// device slots from global index g to the end of the store
u64 dev_room(const tlcg_ctx* c, u64 g) { return c->cap - (g - c->win); }
// the host chunk holding spilled state g (< win)
const tlcg_ctx::HostChunk& chunk_of(const tlcg_ctx* c, u64 g) {
  auto it = std::upper_bound(c->hchunks.begin(), c->hchunks.end(), g,
                             [](u64 x, const tlcg_ctx::HostChunk& h) { return x < h.g0; });
  return *(it - 1);
}

// first unused slot of the state store
u64 store_end(const tlcg_ctx* c) {
  return c->engine != TLCG_ENGINE_GLOBAL ? c->comp_store_used : distinct_of(c);
}

// Pinned host memory for spilled levels.  hipHostMalloc pins 4 KiB pages one
// by one (0.23 s/GiB to allocate, 0.16 s/GiB to free on the MI355X box,
// profiles/r01_pin_probe.jsonl); an anonymous mapping backed by transparent
// huge pages, zeroed by a few threads and then registered with HIP, is ready
// 30x sooner and copies at the same 57 GB/s.  Blocks are pooled across runs.
void* host_block(tlcg_ctx* c, size_t bytes) {
  bytes = (bytes + (2u << 20) - 1) & ~(size_t)((2u << 20) - 1);
  size_t best = c->host_pool.size();
  for (size_t i = 0; i < c->host_pool.size(); ++i)
    if (c->host_pool[i].bytes >= bytes && (best == c->host_pool.size() || c->host_pool[i].bytes < c->host_pool[best].bytes))
      best = i;
  if (best < c->host_pool.size()) {
    void* p = c->host_pool[best].p;
    c->host_pool.erase(c->host_pool.begin() + (long)best);
    return p;
  }
  void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
  if (p == MAP_FAILED) return nullptr;
  madvise(p, bytes, MADV_HUGEPAGE);
  const unsigned hw = std::thread::hardware_concurrency();
  const size_t nt = std::max<size_t>(1, std::min<size_t>({16, hw ? hw : 1, bytes >> 26}));
  std::vector<std::thread> th;
  const size_t per = (bytes / nt + 4095) & ~(size_t)4095;
  for (size_t i = 0; i < nt; ++i)
    th.emplace_back([=] {
      const size_t off = i * per;
      if (off < bytes) std::memset((char*)p + off, 0, std::min(per, bytes - off));
    });
  for (auto& t : th) t.join();
  if (hipHostRegister(p, bytes, hipHostRegisterDefault) != hipSuccess) {
    munmap(p, bytes);
    return nullptr;
  }
  c->host_sizes.emplace_back(p, bytes);
  return p;
}

size_t host_block_bytes(const tlcg_ctx* c, void* p) {
  for (const auto& b : c->host_sizes)
    if (b.first == p) return b.second;
  return 0;
}

// back to the pool (the next run reuses it)
void host_release(tlcg_ctx* c, void* p) {
  if (p) c->host_pool.push_back({p, host_block_bytes(c, p)});
}

void free_host_chunks(tlcg_ctx* c) {
  for (auto& h : c->hchunks) {
    host_release(c, h.st);
    host_release(c, h.par);
  }
  c->hchunks.clear();
  c->win = 0;
}

void destroy_host_pool(tlcg_ctx* c) {
  free_host_chunks(c);
  for (const auto& b : c->host_pool) {
    hipHostUnregister(b.p);
    munmap(b.p, b.bytes);
  }
  c->host_pool.clear();
  c->host_sizes.clear();
}

bool alloc_bytes(tlcg_ctx* c, void** p, size_t bytes, const char* what) {
  hipError_t e = hipMalloc(p, bytes);
  if (e != hipSuccess) {
    char b[256];
    std::snprintf(b, sizeof b, "out of device memory allocating %s (%.2f GiB): %s", what,
                  bytes / 1073741824.0, hipGetErrorString(e));
    c->err = b;
    *p = nullptr;
    return false;
  }
  return true;
}

// Spill: move the committed states [win, f0) -- every level below the
// frontier -- to a pinned host chunk, and slide [f0, end) to the start of the
// device store.  Between kernels only (synchronous).
bool spill_below(tlcg_ctx* c, u64 f0, u64 end) {
  const u64 n = f0 - c->win, w = c->words;
  tlcg_ctx::HostChunk h{c->win, n, nullptr, nullptr};
  const bool tr = std::getenv("TLCG_SPILL_TRACE") != nullptr;
  auto t0 = std::chrono::steady_clock::now();
  auto ms = [&]() { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(); };
  h.st = (u64*)host_block(c, n * 8 * w);
  h.par = h.st ? (u64*)host_block(c, n * 8) : nullptr;
  if (!h.par) {
    host_release(c, h.st);
    char b[160];
    std::snprintf(b, sizeof b, "out of pinned host memory spilling %llu states (%.2f GiB)", (unsigned long long)n,
                  n * 8.0 * (w + 1) / 1073741824.0);
    c->err = b;
    return false;
  }
  const double t_alloc = ms();
  HIPCHK(hipMemcpyAsync(h.st, c->d_states, n * 8 * w, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipMemcpyAsync(h.par, c->d_parents, n * 8, hipMemcpyDeviceToHost, c->stream));
  // pieces of at most n states: source and destination never overlap
  for (u64 off = 0; off < end - f0; off += n) {
    const u64 m = std::min<u64>(n, end - f0 - off);
    HIPCHK(hipMemcpyAsync(c->d_states + off * w, c->d_states + (n + off) * w, m * 8 * w, hipMemcpyDeviceToDevice,
                          c->stream));
    HIPCHK(hipMemcpyAsync(c->d_parents + off, c->d_parents + n + off, m * 8, hipMemcpyDeviceToDevice, c->stream));
  }
  HIPCHK(hipStreamSynchronize(c->stream));
  if (tr)
    std::fprintf(stderr, "spill: %llu states, alloc %.1f ms, copies %.1f ms\n", (unsigned long long)n, t_alloc,
                 ms() - t_alloc);
  c->hchunks.push_back(h);
  c->win = f0;
  return true;
}

// grow the state store so that it holds the states up to global index `need`
// (keeps contents); with opts.spill, first spill the levels below the frontier
// when the store would outgrow its budget
bool ensure_store(tlcg_ctx* c, u64 need) {
  if (need - c->win <= c->cap) return true;
  // in use: [win, end) (nothing while a recover loads the store)
  const u64 end = std::max<u64>(c->win, std::min<u64>(c->win + c->cap, store_end(c) + c->pending));
  size_t fr = 0, tot = 0;
  const bool have_fr = hipMemGetInfo(&fr, &tot) == hipSuccess;
  // states the device could hold: free memory (both arrays, old ones freed after the copy) + what it holds
  const u64 room = have_fr ? (u64)(fr * 0.9) / (8 * (c->words + 1)) + c->cap : ~0ull;
  const u64 budget = c->opts.spill && c->opts.device_store_cap ? std::min<u64>(room, c->opts.device_store_cap) : room;
  if (c->opts.spill && c->engine == TLCG_ENGINE_GLOBAL && c->level_base.size() >= 2 && need - c->win > budget) {
    const u64 f0 = c->level_base[c->level_base.size() - 2];  // first state of the frontier
    // worth a pass when it frees at least 1/16 of what stays (bounds the slide's pieces)
    if (f0 > c->win && (f0 - c->win) * 16 >= end - f0) {
      if (!spill_below(c, f0, end)) return false;
      if (need - c->win <= c->cap) return true;
    }
  }
  const u64 dn = need - c->win;
  u64 ncap = std::max<u64>(dn + dn / 4, c->cap * 2);
  ncap = std::max<u64>(ncap, 1u << 16);
  if (ncap > budget && dn <= budget) ncap = budget;
  u64 *ns = nullptr, *np = nullptr;
  if (!alloc_bytes(c, (void**)&ns, ncap * 8 * c->words, "state store")) return false;
  if (!alloc_bytes(c, (void**)&np, ncap * 8, "parent log")) { hipFree(ns); return false; }
  const u64 keep = end - c->win;
  if (keep) {
    HIPCHK(hipMemcpyAsync(ns, c->d_states, keep * 8 * c->words, hipMemcpyDeviceToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(np, c->d_parents, keep * 8, hipMemcpyDeviceToDevice, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
  }
  hipFree(c->d_states);
  hipFree(c->d_parents);
  c->d_states = ns;
  c->d_parents = np;
  c->cap = ncap;
  return true;
}

// Calls fn(dev, m) on the stored states [g0, g1) in order, m at a time: the
// device window in place, spilled ranges through a device staging buffer.
// fn enqueues on the context's stream and returns false on a launch error.
template <typename F>
bool for_each_stored(tlcg_ctx* c, u64 g0, u64 g1, F&& fn) {
  const u64 w = c->words;
  const u64 e = std::min(g1, c->win);
  if (g0 < e) {
    const u64 stage_n = 1u << 22;
    u64* stage = nullptr;
    if (!alloc_bytes(c, (void**)&stage, stage_n * 8 * w, "host-store staging")) return false;
    bool ok = true;
    for (u64 g = g0; ok && g < e;) {
      const auto& h = chunk_of(c, g);
      const u64 m = std::min<u64>(std::min<u64>(stage_n, e - g), h.g0 + h.n - g);
      ok = hipMemcpyAsync(stage, h.st + (g - h.g0) * w, m * 8 * w, hipMemcpyHostToDevice, c->stream) == hipSuccess &&
           fn((const u64*)stage, m) && hipStreamSynchronize(c->stream) == hipSuccess;
      g += m;
    }
    hipFree(stage);
    if (!ok) {
      c->err = "reading spilled states back failed";
      return false;
    }
  }
  const u64 a = std::max(g0, c->win);
  if (a < g1 && !fn((const u64*)dev_state(c, a), g1 - a)) {
    c->err = "kernel launch failed";
    return false;
  }
  return true;
}

// (re)build the FPSet at 2^log2 slots holding the stored states [t0_base, n)
// (with the host FPSet tier, older states are in the host runs)
bool rebuild_fpset(tlcg_ctx* c, int log2, u64 n) {
  if (log2 != c->log2 || !c->d_slots || (c->opts.tlc_order && !c->d_dkey_slot)) {
    hipFree(c->d_slots);
    c->d_slots = nullptr;
    hipFree(c->d_dkey_slot);
    c->d_dkey_slot = nullptr;
    if (!alloc_bytes(c, (void**)&c->d_slots, ((8ull * c->words) << log2), "FPSet")) return false;
    if (c->opts.tlc_order && !alloc_bytes(c, (void**)&c->d_dkey_slot, (8ull << log2), "FPSet discovery keys"))
      return false;
    c->log2 = log2;
  }
  HIPCHK(hipMemsetAsync(c->d_slots, 0, (8ull * c->words) << log2, c->stream));
  if (c->d_dkey_slot) HIPCHK(hipMemsetAsync(c->d_dkey_slot, 0xFF, 8ull << log2, c->stream));
  if (n > c->t0_base) {
    HIPCHK(hipMemsetAsync(c->d_aux, 0, sizeof(LevelCtr), c->stream));
    auto reinsert = [&](const u64* dev, u64 m) {
      if (c->words == 1)
        k_reinsert<u64><<<grid_for(m, BLOCK, 0x7fffffffu), BLOCK, 0, c->stream>>>(dev, m, c->d_slots, log2, c->d_aux);
      else
        k_reinsert<u128><<<grid_for(m, BLOCK, 0x7fffffffu), BLOCK, 0, c->stream>>>((const u128*)dev, m, c->d_slots,
                                                                                  log2, c->d_aux);
      return hipGetLastError() == hipSuccess;
    };
    if (!for_each_stored(c, c->t0_base, n, reinsert)) return false;
    HIPCHK(hipMemcpyAsync(c->h_aux, c->d_aux, sizeof(LevelCtr), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    if (c->h_aux->overflow) {
      c->err = "FPSet rebuild overflowed";
      return false;
    }
  }
  return true;
}

// ---- host FPSet tier (opts.fpset_spill; TLC's DiskFPSet) ----

double wall_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// largest HBM table: the option, else what free memory allows
int fpset_max_log2(tlcg_ctx* c) {
  if (c->opts.log2_fpset_max > 0) return c->opts.log2_fpset_max;
  if (c->opts.log2_fpset_slots > 0) return c->opts.log2_fpset_slots;
  size_t fr = 0, tot = 0;
  if (hipMemGetInfo(&fr, &tot) != hipSuccess) return 40;
  const u64 avail = (u64)(fr * 0.8) + (c->d_slots ? (8ull * c->words) << c->log2 : 0);
  const u64 per_slot = 8ull * c->words + (c->opts.tlc_order ? 8 : 0);
  int l = 16;
  while (l < 40 && (per_slot << (l + 1)) <= avail) ++l;
  return l;
}

void free_tier(tlcg_ctx* c) {
  for (auto& r : c->runs) host_release(c, r.keys);
  c->runs.clear();
  c->t0_base = 0;
  c->tier_queued = c->tier_dups = 0;
  for (double& t : c->tier_ms) t = 0;
  if (c->d_bloom) (void)hipMemsetAsync(c->d_bloom, 0, 64ull << c->bloom_log2, c->stream);
}

// insert every host run's keys into a (new) Bloom filter of 2^log2b blocks
bool bloom_rebuild(tlcg_ctx* c, int log2b) {
  u64* nb = nullptr;
  if (!alloc_bytes(c, (void**)&nb, 64ull << log2b, "FPSet tier Bloom filter")) return false;
  hipFree(c->d_bloom);
  c->d_bloom = nb;
  c->bloom_log2 = log2b;
  HIPCHK(hipMemsetAsync(c->d_bloom, 0, 64ull << log2b, c->stream));
  const u64 stage_n = 1u << 24;
  u64* stage = nullptr;
  bool ok = true;
  for (const auto& r : c->runs)
    for (u64 off = 0; ok && off < r.n; off += stage_n) {
      if (!stage && !alloc_bytes(c, (void**)&stage, stage_n * 8, "Bloom staging")) return false;
      const u64 m = std::min<u64>(stage_n, r.n - off);
      ok = hipMemcpyAsync(stage, r.keys + off, m * 8, hipMemcpyHostToDevice, c->stream) == hipSuccess;
      k_bloom_insert<<<grid_for(m, BLOCK, 0x7fffffffu), BLOCK, 0, c->stream>>>(stage, m, c->d_bloom, log2b);
      ok = ok && hipGetLastError() == hipSuccess && hipStreamSynchronize(c->stream) == hipSuccess;
    }
  hipFree(stage);
  if (!ok) c->err = "Bloom filter rebuild failed";
  return ok;
}

// Merge every host run into one sorted run (lookups cost a search per run).
// Keys are uniform on [0, 2^64): thread t merges the key range
// [t, t + 1) * 2^64 / T of all runs into its own slice of the output.
constexpr size_t kMaxRuns = 16;

bool merge_runs(tlcg_ctx* c) {
  u64 total = 0;
  for (const auto& r : c->runs) total += r.n;
  u64* out = (u64*)host_block(c, total * 8);
  if (!out) {
    c->err = "out of host memory merging the FPSet tier";
    return false;
  }
  const unsigned hw = std::thread::hardware_concurrency();
  const u64 nt = std::max<u64>(1, std::min<u64>(16, hw ? hw : 1));
  const size_t R = c->runs.size();
  // cut[t][r]: first index of run r in thread t's key range
  std::vector<std::vector<u64>> cut(nt + 1, std::vector<u64>(R));
  for (u64 t = 0; t <= nt; ++t)
    for (size_t r = 0; r < R; ++r) {
      const auto& run = c->runs[r];
      cut[t][r] = t == nt ? run.n
                          : t == 0 ? 0
                                   : (u64)(std::lower_bound(run.keys, run.keys + run.n,
                                                            (u64)(((unsigned __int128)t << 64) / nt)) - run.keys);
    }
  auto work = [&](u64 t) {
    u64 o = 0;
    for (size_t r = 0; r < R; ++r) o += cut[t][r];
    u64* base = out + o;
    u64 len = 0;
    for (size_t r = 0; r < R; ++r) {  // append run r's piece, then merge it into what is there
      const u64 a = cut[t][r], b = cut[t + 1][r];
      std::memcpy(base + len, c->runs[r].keys + a, (b - a) * 8);
      std::inplace_merge(base, base + len, base + len + (b - a));
      len += b - a;
    }
  };
  std::vector<std::thread> th;
  for (u64 t = 1; t < nt; ++t) th.emplace_back(work, t);
  work(0);
  for (auto& t : th) t.join();
  for (auto& r : c->runs) host_release(c, r.keys);
  c->runs.assign(1, tlcg_ctx::Run{out, total});
  return true;
}

// Move the stored states [t0_base, g1) out of the HBM table into a new
// sorted host run.  The sort reuses the table's own memory (the table is
// rebuilt right after): keys and their alternate buffer fit in its 8 * 2^log2
// bytes because its load is <= 1/2.
bool flush_tier(tlcg_ctx* c, u64 g1) {
  const u64 n = g1 - c->t0_base;
  if (!n) return true;
  const double t0 = wall_ms();
  struct Acc {
    double& a;
    double t0;
    ~Acc() { a += wall_ms() - t0; }
  } acc{c->tier_ms[0], t0};
  const u64 half = (1ull << c->log2) / 2;
  if (!c->d_slots || n > half) {
    c->err = "internal: FPSet tier flush larger than the table";
    return false;
  }
  u64* keys = c->d_slots;
  u64* alt = c->d_slots + half;
  u64 off = 0;
  auto mix = [&](const u64* dev, u64 m) {
    k_mix_keys<<<grid_for(m, BLOCK, 0x7fffffffu), BLOCK, 0, c->stream>>>(dev, m, keys + off);
    off += m;
    return hipGetLastError() == hipSuccess;
  };
  if (!for_each_stored(c, c->t0_base, g1, mix)) return false;
  hipcub::DoubleBuffer<u64> db(keys, alt);
  size_t tmp = 0;
  HIPCHK(hipcub::DeviceRadixSort::SortKeys(nullptr, tmp, db, (int)n, 0, 64, c->stream));
  void* d_tmp = nullptr;
  if (!alloc_bytes(c, &d_tmp, tmp, "FPSet tier sort scratch")) return false;
  const hipError_t e = hipcub::DeviceRadixSort::SortKeys(d_tmp, tmp, db, (int)n, 0, 64, c->stream);
  tlcg_ctx::Run r{(u64*)host_block(c, n * 8), n};
  bool ok = e == hipSuccess && r.keys &&
            hipMemcpyAsync(r.keys, db.Current(), n * 8, hipMemcpyDeviceToHost, c->stream) == hipSuccess &&
            hipStreamSynchronize(c->stream) == hipSuccess;
  if (!ok) {
    hipFree(d_tmp);
    host_release(c, r.keys);
    c->err = r.keys ? "FPSet tier flush failed" : "out of host memory for the FPSet tier";
    return false;
  }
  // the Bloom filter: 16+ bits per host-tier state, doubled ahead of need;
  // a resize re-inserts the older runs from host memory, the new run's keys
  // go in from the device copy still at hand
  int lb = std::max(c->bloom_log2, 10);
  while ((512ull << lb) < 16 * g1) ++lb;
  if (lb != c->bloom_log2 || !c->d_bloom) {
    hipFree(d_tmp);
    d_tmp = nullptr;
    if (!bloom_rebuild(c, std::min(lb + 1, 40))) {
      host_release(c, r.keys);
      return false;
    }
  }
  k_bloom_insert<<<grid_for(n, BLOCK, 0x7fffffffu), BLOCK, 0, c->stream>>>(db.Current(), n, c->d_bloom,
                                                                           c->bloom_log2);
  ok = hipGetLastError() == hipSuccess && hipStreamSynchronize(c->stream) == hipSuccess;
  hipFree(d_tmp);
  if (!ok) {
    host_release(c, r.keys);
    c->err = "Bloom filter insert failed";
    return false;
  }
  c->runs.push_back(r);
  c->t0_base = g1;
  return c->runs.size() <= kMaxRuns || merge_runs(c);
}

// first index in [from, n) whose key is >= key, galloping from `from`
inline u64 gallop_lb(const u64* k, u64 n, u64 from, u64 key) {
  if (from >= n || k[from] >= key) return from;
  u64 lo = from, step = 1;  // k[lo] < key
  while (lo + step < n && k[lo + step] < key) {
    lo += step;
    step <<= 1;
  }
  return (u64)(std::lower_bound(k + lo + 1, k + std::min<u64>(n, lo + step + 1), key) - k);
}

// dup[j] = 1 iff the host runs hold key q[j].  The queries are sorted, so
// each thread merges its slice against every run, galloping forward: the
// runs are streamed, not probed at random.  Up to 16 threads.
void host_tier_lookup(const tlcg_ctx* c, const u64* q, u64 m, unsigned char* dup) {
  const unsigned hw = std::thread::hardware_concurrency();
  const u64 nt = std::max<u64>(1, std::min<u64>(std::min<u64>(16, hw ? hw : 1), m / 4096 + 1));
  auto work = [&](u64 a, u64 b) {
    std::memset(dup + a, 0, b - a);
    for (const auto& r : c->runs) {
      u64 pos = (u64)(std::lower_bound(r.keys, r.keys + r.n, q[a]) - r.keys);
      for (u64 j = a; j < b && pos < r.n; ++j) {
        if (dup[j]) continue;
        pos = gallop_lb(r.keys, r.n, pos, q[j]);
        if (pos < r.n && r.keys[pos] == q[j]) dup[j] = 1;
      }
    }
  };
  std::vector<std::thread> th;
  for (u64 t = 1; t < nt; ++t) th.emplace_back(work, m * t / nt, m * (t + 1) / nt);
  work(0, m / nt);
  for (auto& t : th) t.join();
}

// Drop from the level being built, [d, d + n_new) in the device window, the
// states the host runs already hold (stable: TLC order survives).  Returns
// the new count, or ~0 on error.
u64 tier_filter_level(tlcg_ctx* c, u64 d, u64 n_new) {
  if (c->runs.empty() || !n_new) return n_new;
  if (n_new > c->filt_cap) {
    hipFree(c->d_q); hipFree(c->d_keep); hipFree(c->d_sel); hipFree(c->d_ftmp); hipFree(c->d_qn);
    c->d_q = c->d_sel = nullptr;
    c->d_keep = nullptr;
    c->d_ftmp = nullptr;
    c->d_qn = nullptr;
    c->filt_cap = 0;
    const u64 cap = std::max<u64>(n_new + n_new / 4, 1u << 16);
    size_t t1 = 0, t2 = 0;
    if (hipcub::DeviceRadixSort::SortPairs(nullptr, t1, (const u64*)nullptr, (u64*)nullptr, (const u64*)nullptr,
                                           (u64*)nullptr, (int)cap, 0, 64, c->stream) != hipSuccess ||
        hipcub::DeviceSelect::Flagged(nullptr, t2, (const u64*)nullptr, (const unsigned char*)nullptr, (u64*)nullptr,
                                      (unsigned long long*)nullptr, (int)cap, c->stream) != hipSuccess)
      return ~0ull;
    c->ftmp_bytes = std::max(t1, t2);
    if (!alloc_bytes(c, (void**)&c->d_q, cap * 8 * 4, "FPSet tier queue") ||
        !alloc_bytes(c, (void**)&c->d_keep, cap, "FPSet tier flags") ||
        !alloc_bytes(c, (void**)&c->d_sel, cap * 8, "FPSet tier select") ||
        !alloc_bytes(c, &c->d_ftmp, c->ftmp_bytes, "FPSet tier scratch") ||
        !alloc_bytes(c, (void**)&c->d_qn, 16, "FPSet tier counter"))
      return ~0ull;
    c->filt_cap = cap;
  }
  const u64 cap = c->filt_cap;
  u64 *q_key = c->d_q, *q_pos = c->d_q + cap, *q_key2 = c->d_q + 2 * cap, *q_pos2 = c->d_q + 3 * cap;
  u64* lvl = dev_state(c, d);
  double t0 = wall_ms();
  HIPCHK_U(hipMemsetAsync(c->d_qn, 0, 16, c->stream));
  k_tier_filter<<<grid_for(n_new, BLOCK, 0x7fffffffu), BLOCK, 0, c->stream>>>(lvl, n_new, c->d_bloom, c->bloom_log2,
                                                                              q_key, q_pos, c->d_qn);
  HIPCHK_U(hipGetLastError());
  unsigned long long m = 0;
  HIPCHK_U(hipMemcpyAsync(&m, c->d_qn, 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK_U(hipStreamSynchronize(c->stream));
  c->tier_queued += m;
  c->tier_ms[1] += wall_ms() - t0;
  t0 = wall_ms();
  if (!m) return n_new;
  // sorted queries walk the runs in order
  size_t tmp = c->ftmp_bytes;
  HIPCHK_U(hipcub::DeviceRadixSort::SortPairs(c->d_ftmp, tmp, q_key, q_key2, q_pos, q_pos2, (int)m, 0, 64, c->stream));
  std::vector<u64> hq(m);
  std::vector<unsigned char> dup(m);
  HIPCHK_U(hipMemcpyAsync(hq.data(), q_key2, m * 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK_U(hipStreamSynchronize(c->stream));
  host_tier_lookup(c, hq.data(), m, dup.data());
  u64 ndup = 0;
  for (u64 j = 0; j < m; ++j) ndup += dup[j];
  c->tier_dups += ndup;
  c->tier_ms[2] += wall_ms() - t0;
  t0 = wall_ms();
  if (!ndup) return n_new;
  unsigned char* d_dup = (unsigned char*)q_key;  // the unsorted keys are no longer needed
  HIPCHK_U(hipMemcpyAsync(d_dup, dup.data(), m, hipMemcpyHostToDevice, c->stream));
  HIPCHK_U(hipMemsetAsync(c->d_keep, 1, n_new, c->stream));
  k_tier_mark<<<grid_for(m, BLOCK, 0x7fffffffu), BLOCK, 0, c->stream>>>(q_pos2, d_dup, m, c->d_keep);
  HIPCHK_U(hipGetLastError());
  // compact states and parent refs in place, keeping their order
  unsigned long long kept = 0;
  u64* arrays[2] = {lvl, dev_parent(c, d)};
  for (u64* arr : arrays) {
    tmp = c->ftmp_bytes;
    HIPCHK_U(hipcub::DeviceSelect::Flagged(c->d_ftmp, tmp, arr, c->d_keep, c->d_sel, c->d_qn, (int)n_new, c->stream));
    HIPCHK_U(hipMemcpyAsync(arr, c->d_sel, n_new * 8, hipMemcpyDeviceToDevice, c->stream));
  }
  HIPCHK_U(hipMemcpyAsync(&kept, c->d_qn, 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK_U(hipStreamSynchronize(c->stream));
  c->tier_ms[3] += wall_ms() - t0;
  if (kept != n_new - ndup) {
    c->err = "internal: FPSet tier compaction count";
    return ~0ull;
  }
  return kept;
}

// The host tier's flush point: a level boundary, keeping the newest levels
// (up to 4) in the HBM table when the table still fits `need` (a global index
// end) under its cap -- most rediscovered states are a few levels old, and
// those then never reach the host lookup.
u64 tier_flush_point(tlcg_ctx* c, u64 need, int max_log2) {
  const u64 d = distinct_of(c);
  const size_t nl = c->level_base.size();
  for (int keep = 4; keep > 0; --keep) {
    if ((size_t)keep >= nl) continue;
    const u64 g = c->level_base[nl - 1 - (size_t)keep];
    if (g > c->t0_base && g < d && 2 * (need - g) <= (1ull << max_log2)) return g;
  }
  return d;
}

// keep the HBM table's load <= 1/2 for `need` states (a global index end):
// grow it, or with the host tier move its older states to the host first
bool ensure_fpset(tlcg_ctx* c, u64 need) {
  auto size_for = [&](u64 n0) {
    int l = std::max(c->log2, c->opts.fpset_spill ? 10 : 16);
    while ((1ull << l) < 2 * n0 && l < 40) ++l;
    return l;
  };
  int l = size_for(need - c->t0_base);
  if (c->d_slots && l == c->log2) return true;
  const int mx = c->opts.fpset_spill ? fpset_max_log2(c) : 40;
  if (c->opts.fpset_spill && l > mx && distinct_of(c) > c->t0_base) {
    if (!flush_tier(c, tier_flush_point(c, need, mx))) return false;
    l = size_for(need - c->t0_base);
  }
  return rebuild_fpset(c, l, distinct_of(c) + c->pending);
}

// after an FPSet overflow: grow the table, or flush it to the host tier
bool regrow_fpset(tlcg_ctx* c, unsigned ovf, u64 n) {
  if (!(ovf & OVF_FPSET)) return rebuild_fpset(c, c->log2, n);
  const u64 d = distinct_of(c);
  const int mx = c->opts.fpset_spill ? fpset_max_log2(c) : 40;
  if (c->opts.fpset_spill && c->log2 + 1 > mx && d > c->t0_base) {
    if (!flush_tier(c, d)) return false;
    return rebuild_fpset(c, c->log2, n);
  }
  return rebuild_fpset(c, c->log2 + 1, n);
}

bool ensure_scratch(tlcg_ctx* c, u64 n) {
  if (!c->opts.tlc_order || n <= c->scratch_cap) return true;
  u64 ncap = std::max<u64>(n + n / 4, 1u << 16);
  hipFree(c->d_slot_new); hipFree(c->d_dk); hipFree(c->d_dk2); hipFree(c->d_st2); hipFree(c->d_sort_tmp);
  c->d_slot_new = c->d_dk = c->d_dk2 = c->d_st2 = nullptr;
  c->d_sort_tmp = nullptr;
  c->scratch_cap = 0;
  if (!alloc_bytes(c, (void**)&c->d_slot_new, ncap * 8, "TLC-order scratch")) return false;
  if (!alloc_bytes(c, (void**)&c->d_dk, ncap * 8, "TLC-order scratch")) return false;
  if (!alloc_bytes(c, (void**)&c->d_dk2, ncap * 8, "TLC-order scratch")) return false;
  if (!alloc_bytes(c, (void**)&c->d_st2, ncap * 8 * c->words, "TLC-order scratch")) return false;
  size_t tmp = 0;
  const int nmax = (int)std::min<u64>(ncap, 0x7fffffffull);
  if (c->words == 1)
    HIPCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, (const u64*)nullptr, (u64*)nullptr, (const u64*)nullptr,
                                              (u64*)nullptr, nmax, 0, 64, c->stream));
  else
    HIPCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, (const u64*)nullptr, (u64*)nullptr, (const u128*)nullptr,
                                              (u128*)nullptr, nmax, 0, 64, c->stream));
  if (!alloc_bytes(c, &c->d_sort_tmp, tmp, "sort scratch")) return false;
  c->sort_tmp_bytes = tmp;
  c->scratch_cap = ncap;
  return true;
}

bool reset_ctr(tlcg_ctx* c) {
  HIPCHK(hipMemsetAsync(c->d_ctr, 0, sizeof(LevelCtr), c->stream));
  HIPCHK(hipMemsetAsync(&c->d_ctr->event, 0xFF, sizeof(unsigned long long), c->stream));
  return true;
}

bool read_ctr(tlcg_ctx* c) {
  HIPCHK(hipMemcpyAsync(c->h_ctr, c->d_ctr, sizeof(LevelCtr), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return true;
}

void fill_stats(tlcg_ctx* c, tlcg_stats* st) {
  if (!st) return;
  std::memset(st, 0, sizeof *st);
  const bool comp = c->engine != TLCG_ENGINE_GLOBAL;  // an on-chip engine (component, tree)
  const u64 d = comp ? c->comp_distinct : distinct_of(c);
  const int depth = comp ? (int)c->comp_levels.size()
                         : (c->level_base.empty() ? 0 : (int)c->level_base.size() - 1);
  st->generated = comp ? c->comp_generated : c->generated;
  st->distinct = d;
  st->frontier = comp ? (depth ? c->comp_levels[(size_t)depth - 1] : 0)
                      : (depth ? c->level_base[(size_t)depth] - c->level_base[(size_t)depth - 1] : 0);
  st->depth = depth;
  st->engine = (uint64_t)c->engine;
  st->jit_used = (c->jit_used ? 1 : 0) | (c->engine == TLCG_ENGINE_COMPONENT && c->comp_code ? 2 : 0);
  st->host_states = c->engine == TLCG_ENGINE_GLOBAL ? c->win : 0;  // (the component engine's window starts after its records)
  st->fpset_host_states = c->t0_base;
  if (std::getenv("TLCG_TIER_TRACE") && c->opts.fpset_spill)
    std::fprintf(stderr,
                 "tier: host states %llu in %zu runs, queued %llu, dups %llu, table 2^%d; ms flush %.1f "
                 "filter %.1f lookup %.1f compact %.1f\n",
                 (unsigned long long)c->t0_base, c->runs.size(), (unsigned long long)c->tier_queued,
                 (unsigned long long)c->tier_dups, c->log2, c->tier_ms[0], c->tier_ms[1], c->tier_ms[2],
                 c->tier_ms[3]);
  st->status = c->status;
  st->invariant = -1;
  st->action = -1;
  st->event_gidx = c->ev_parent_gidx;
  if (c->ev_word != NO_EVENT) {
    const int kind = (int)((c->ev_word >> 4) & 3);
    if (kind == EVK_VIOLATION || kind == EVK_INV_ERROR) st->invariant = (int)(c->ev_word & 15);
    st->action = c->ev_action;
  }
  const double g = (double)st->generated, n = (double)d;
  st->fp_collision_optimistic = n * (g - n) / 18446744073709551616.0;
  st->kernel_ms = c->kernel_ms;
  st->expand_ms = c->expand_ms;
  st->levels_redone = c->levels_redone;
  // the trace and tlcg_tlc_stop_stats are TLC -workers 1's: a TLC-order run,
  // or an on-chip engine's error on a closed partition (one rank)
  st->tlc_exact = c->status >= TLCG_VIOLATION && c->opts.world == 1 &&
                  ((c->engine == TLCG_ENGINE_GLOBAL && c->opts.tlc_order) || c->stop_cached ||
                   (c->engine != TLCG_ENGINE_GLOBAL && !c->hm.L.producer && c->ev_comp != ~0ull));
}

// the state word of store slot g holding a component code (the tree's closed
// mode): chunk g / cap is the component of initial state tree_r0 + g / cap
u128 tree_code_word(const tlcg_ctx* c, u64 g, uint32_t code) {
  const Layout& L = c->hm.L;
  const u128 s0 = init_state<u128>(L, c->tree_r0 + g / (u64)c->tree_cap);
  const CodeConsts kc = code_consts(L, comp_msgs_init(L, (u64)s0));
  return code_word<u128>(L, kc, s0 & messages_mask<u128>(L), code);
}

// the component-engine pass whose store holds 32-bit records (comp_record)
// at slot g, or null
const tlcg_ctx::CompPass* comp_code_pass(const tlcg_ctx* c, u64 g) {
  if (c->engine != TLCG_ENGINE_COMPONENT) return nullptr;
  for (const auto& ps : c->passes)
    if (ps.codes && g >= ps.store_base && g < ps.store_base + component_store_slots(ps.n, ps.K)) return &ps;
  return nullptr;
}

// the state word and parent reference of slot g of such a pass, from its
// record: the slot names the batch, queue position and lane, so the lane's
// component (its `messages` and code constants) and the parent's slot
u64 comp_slot_decode(const tlcg_ctx* c, const tlcg_ctx::CompPass& ps, u64 g, uint32_t rec, u64* p) {
  const Layout& L = c->hm.L;
  const u64 off = g - ps.store_base, row = (u64)ps.K * 64;
  const u64 b = off / row, lane = off % 64;
  const u64 pos = off % row / 64, ci = b * 64 + lane;
  const u64 idx0 = ps.list.empty() ? ps.r0 + ci : ps.list[ci] & ((1ull << 40) - 1);
  const u64 s0 = init_state(L, idx0);
  const CodeConsts kc = code_consts(L, comp_msgs_init(L, s0));
  const int mb = L.msg_sh + L.N * L.mw;
  if (p) {
    const u64 gp = ps.store_base + b * row + ((rec >> 16) & 255) * 64 + lane;
    *p = pos == 0 ? NO_PARENT
                  : ((u64)c->opts.rank << 56) | (gp << L.ord_bits) | (u64)ordinal_of(L, (int)(rec >> 24), 0);
  }
  return (s0 & L.msgs_mask) | ((u64)code_decode(L, kc, (ckey)(rec & 0xFFFF)) << mb);
}

bool state_at(tlcg_ctx* c, u64 g, u128* s, u64* p) {
  if (const tlcg_ctx::CompPass* ps = comp_code_pass(c, g)) {
    uint32_t rec = 0;
    HIPCHK(hipMemcpy(&rec, c->d_crec + (g - ps->store_base), 4, hipMemcpyDeviceToHost));
    *s = comp_slot_decode(c, *ps, g, rec, p);
    return true;
  }
  if (c->tree_codes) {
    uint32_t code = 0;
    HIPCHK(hipMemcpy(&code, reinterpret_cast<const uint32_t*>(c->d_states) + g, 4, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(p, dev_parent(c, g), 8, hipMemcpyDeviceToHost));
    *s = tree_code_word(c, g, code);
    return true;
  }
  uint64_t w[2] = {0, 0};
  if (g < c->win) {
    const auto& h = chunk_of(c, g);
    std::memcpy(w, h.st + (g - h.g0) * c->words, 8 * c->words);
    *p = h.par[g - h.g0];
  } else {
    HIPCHK(hipMemcpy(w, dev_state(c, g), 8 * c->words, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(p, dev_parent(c, g), 8, hipMemcpyDeviceToHost));
  }
  *s = join_words(w, c->words);
  return true;
}

// successor at a Next ordinal of a state held as u128 (either width)
int successor_at_any(const tlcg_ctx* c, u128 s, int ord, u128* t) {
  if (c->words == 2) return successor_at<u128>(c->hm.L, s, ord, t);
  u64 t1 = 0;
  const int r = successor_at<u64>(c->hm.L, (u64)s, ord, &t1);
  *t = t1;
  return r;
}

// Interpret the level's event word (world == 1 or a local event).
bool resolve_event(tlcg_ctx* c, u64 ev, int level) {
  const Layout& L = c->hm.L;
  c->ev_word = ev;
  c->ev_level = level;
  const int kind = (int)((ev >> 4) & 3);
  const int index = (int)(ev & 15);
  const u64 dkey = ev >> 6;
  switch (kind) {
    case EVK_VIOLATION: c->status = TLCG_VIOLATION; break;
    case EVK_INV_ERROR: c->status = TLCG_INVARIANT_ERROR; break;
    case EVK_DEADLOCK: c->status = TLCG_DEADLOCK; break;
    default: c->status = TLCG_ACTION_ERROR; break;
  }
  if (level == 0) {  // an initial state (dkey = enumeration index)
    c->ev_state = c->words == 2 ? init_state<u128>(L, dkey) : (u128)init_state<u64>(L, dkey);
    c->ev_parent_gidx = NO_PARENT;
    c->ev_action = TLCG_ACT_INIT;
    return true;
  }
  if (((dkey >> 50) & 3) == 1) {  // a state absorbed from another rank (k_user_check): its store index
    u128 s = 0;
    u64 p = 0;
    if (!state_at(c, dkey & ((1ull << 50) - 1), &s, &p)) return false;
    c->ev_state = s;
    c->ev_parent_ref = p;
    c->ev_parent_gidx = NO_PARENT;
    c->ev_action = action_of_ordinal(L, (int)(p & ((1ull << L.ord_bits) - 1)));
    return true;
  }
  if ((dkey >> 51) & 1) {  // a state absorbed from another rank: inbox position
    const u64 i = dkey & ((1ull << 51) - 1);
    u64 rec[2];
    HIPCHK(hipMemcpy(rec, c->d_inbox + 2 * i, 16, hipMemcpyDeviceToHost));
    c->ev_state = rec[0];
    c->ev_parent_ref = rec[1];
    c->ev_parent_gidx = NO_PARENT;
    c->ev_action = action_of_ordinal(L, (int)(rec[1] & ((1ull << L.ord_bits) - 1)));
    return true;
  }
  const u64 pg = dkey >> L.ord_bits;
  const int ord = (int)(dkey & ((1ull << L.ord_bits) - 1));
  u128 ps = 0;
  u64 pp = 0;
  if (!state_at(c, pg, &ps, &pp)) return false;
  c->ev_parent_gidx = pg;
  c->ev_parent_ref = ((u64)c->opts.rank << 56) | dkey;
  if (kind == EVK_DEADLOCK) {
    c->ev_state = ps;
    c->ev_action = -1;
  } else if (kind == EVK_ACTION_ERROR) {
    c->ev_state = ps;
    c->ev_action = index;
  } else {
    u128 t = 0;
    if (successor_at_any(c, ps, ord, &t) != 1) {
      c->err = "internal: violating successor could not be re-derived";
      return false;
    }
    c->ev_state = t;
    c->ev_action = action_of_ordinal(L, ord);
  }
  return true;
}


// Locate a component-engine event (component.h's key) in the store.
bool resolve_comp_event(tlcg_ctx* c, u64 ev) {
  const Layout& L = c->hm.L;
  const int level = (int)(ev >> 56);
  const u64 idx0 = (ev >> 20) & ((1ull << 36) - 1);
  const int pos = (int)((ev >> 12) & 255);
  const int action = (int)((ev >> 8) & 15);
  const int kind = (int)((ev >> 4) & 3);
  c->ev_word = ev;
  c->ev_level = level;
  c->ev_comp = idx0;
  switch (kind) {
    case EVK_VIOLATION: c->status = TLCG_VIOLATION; break;
    case EVK_INV_ERROR: c->status = TLCG_INVARIANT_ERROR; break;
    case EVK_DEADLOCK: c->status = TLCG_DEADLOCK; break;
    default: c->status = TLCG_ACTION_ERROR; break;
  }
  if (level == 0) {  // an initial state
    c->ev_state = init_state(L, idx0);
    c->ev_parent_gidx = NO_PARENT;
    c->ev_action = TLCG_ACT_INIT;
    return true;
  }
  // which pass completed this component, and its slot there
  u64 gidx = NO_PARENT;
  for (const auto& ps : c->passes) {
    u64 ci = NO_PARENT;
    if (ps.list.empty()) {
      if (idx0 >= ps.r0 && idx0 < ps.r0 + ps.n) ci = idx0 - ps.r0;
    } else {
      for (u64 i = 0; i < ps.list.size(); ++i)
        if ((ps.list[i] & ((1ull << 40) - 1)) == idx0) ci = i;  // entries carry counted levels above bit 40
    }
    if (ci != NO_PARENT) gidx = ps.store_base + (ci / 64) * (u64)ps.K * 64 + (u64)pos * 64 + (ci % 64);
  }
  if (gidx == NO_PARENT) {
    c->err = "internal: component of the event not found";
    return false;
  }
  u128 ps = 0;
  u64 pp = 0;
  if (!state_at(c, gidx, &ps, &pp)) return false;
  c->ev_parent_gidx = gidx;
  c->ev_parent_ref = ((u64)c->opts.rank << 56) | (gidx << L.ord_bits);
  if (kind == EVK_DEADLOCK) {
    c->ev_state = ps;
    c->ev_action = -1;
  } else if (kind == EVK_ACTION_ERROR) {
    c->ev_state = ps;
    c->ev_action = action;
  } else {
    u128 t = 0;
    if (successor_at_any(c, ps, ordinal_of(L, action, 0), &t) != 1) {
      c->err = "internal: violating successor could not be re-derived";
      return false;
    }
    c->ev_state = t;
    c->ev_action = action;
  }
  return true;
}

// ---- TLC's one-worker run on one component of a closed partition ----
//
// Without a Producer the reachable graph is the disjoint union of one
// component per initial state, and TLC's FIFO queue holds every level in the
// Init order of the components, then each component's own FIFO order (level
// 0 is in Init order and successors never leave their component).  So TLC's
// first error lies in the least component with an error at the least error
// level E, and is that component's own first error: the host replays just
// that component (<= a few thousand states) in TLC's worker order
// (ModelChecker.doNext, [TLC-ext]: FIFO states, Next disjuncts in order, each
// action's successors counted before any is checked, the run stopping at the
// first violating new state, a failing action or after a deadlocked state's
// actions), which gives the trace and the component's share of TLC's stop
// counters.  The on-chip engines then report TLC's error without a
// global-engine re-run.
struct CompReplay {
  int status = TLCG_DONE, invariant = -1, action = -1, kind = -1;
  int level = -1;              // E: the violating state's level, or the failing / deadlocked state's + 1
  std::vector<u128> trace;     // Init .. the violating (or the failing) state
  std::vector<int> acts;
  u64 p_index = 0;             // the stopping state p's position in the component's level E - 1
  u64 outdeg_before = 0;       // out-degrees of the component's level-(E - 1) states before p
  u64 partial = 0;             // p's successors counted before the stop
  u64 found_next = 0;          // the component's level-E states discovered by the stop (the violating one too)
};

int check_any(const tlcg_ctx* c, u128 s) {
  return c->words == 2 ? host_check_all<u128>(c->hm, s) : host_check_all<u64>(c->hm, (u64)s);
}

// false when the component holds no error (the caller's event was not this component's)
bool replay_component(const tlcg_ctx* c, u64 idx0, CompReplay* out) {
  const Layout& L = c->hm.L;
  struct H {
    size_t operator()(u128 x) const { return (size_t)mix64((u64)x ^ mix64((u64)(x >> 64) + 0x9E3779B97F4A7C15ull)); }
  };
  std::unordered_map<u128, uint32_t, H> seen;
  std::vector<u128> q;
  std::vector<int32_t> par, act, lvl;
  const u128 s0 = c->words == 2 ? init_state<u128>(L, idx0) : (u128)init_state<u64>(L, idx0);
  auto chain = [&](int64_t i, CompReplay* r) {  // Init .. state i
    for (int64_t j = i; j >= 0; j = par[(size_t)j]) {
      r->trace.push_back(q[(size_t)j]);
      r->acts.push_back(par[(size_t)j] < 0 ? TLCG_ACT_INIT : act[(size_t)j]);
    }
    std::reverse(r->trace.begin(), r->trace.end());
    std::reverse(r->acts.begin(), r->acts.end());
  };
  q.push_back(s0);
  par.push_back(-1);
  act.push_back(TLCG_ACT_INIT);
  lvl.push_back(0);
  seen.emplace(s0, 0u);
  const int c0 = check_any(c, s0);
  if (c0 >= 0) {
    out->status = (c0 & 1) ? TLCG_INVARIANT_ERROR : TLCG_VIOLATION;
    out->kind = (c0 & 1) ? EVK_INV_ERROR : EVK_VIOLATION;
    out->invariant = c0 >> 1;
    out->action = TLCG_ACT_INIT;
    out->level = 0;
    chain(0, out);
    return true;
  }
  const int nord = L.nkv + N_ACTIONS - 1;  // Next ordinals (compaction.tla:216-231)
  int64_t lvl_start = 0, cur_level = 0;
  u64 outdeg_sum = 0, next_found = 0;
  for (size_t head = 0; head < q.size(); ++head) {
    const u128 p = q[head];
    if (lvl[head] != cur_level) {  // a new level is dequeued
      cur_level = lvl[head];
      lvl_start = (int64_t)head;
      outdeg_sum = 0;
      next_found = 0;
    }
    u64 gen = 0;
    auto stop = [&](int status, int kind, int action, int inv, int64_t last) {
      out->status = status;
      out->kind = kind;
      out->action = action;
      out->invariant = inv;
      out->level = (int)cur_level + 1;
      out->p_index = (u64)((int64_t)head - lvl_start);
      out->outdeg_before = outdeg_sum;
      out->partial = gen;
      out->found_next = next_found;
      chain(last, out);
      return true;
    };
    for (int o = 0; o < nord;) {
      // one action's successors: the Producer's (key, value) pairs, or one disjunct
      const int a = action_of_ordinal(L, o);
      const int o1 = a == ACT_PRODUCER ? L.nkv : o + 1;
      std::vector<u128> ts;
      for (; o < o1; ++o) {
        u128 t = 0;
        const int r = successor_at_any(c, p, o, &t);
        if (r == 2) return stop(TLCG_ACTION_ERROR, EVK_ACTION_ERROR, a, -1, (int64_t)head);
        if (r == 1) ts.push_back(t);
      }
      gen += ts.size();  // counted as one StateVec before any is put and checked
      for (const u128 t : ts) {
        if (seen.count(t)) continue;
        seen.emplace(t, (uint32_t)q.size());
        q.push_back(t);
        par.push_back((int32_t)head);
        act.push_back(a);
        lvl.push_back((int32_t)cur_level + 1);
        ++next_found;
        const int ci = check_any(c, t);
        if (ci >= 0)
          return stop((ci & 1) ? TLCG_INVARIANT_ERROR : TLCG_VIOLATION, (ci & 1) ? EVK_INV_ERROR : EVK_VIOLATION,
                       a, ci >> 1, (int64_t)q.size() - 1);
      }
    }
    if (!gen && L.check_deadlock) return stop(TLCG_DEADLOCK, EVK_DEADLOCK, -1, -1, (int64_t)head);
    outdeg_sum += gen;
    if (q.size() > (1u << 24)) return false;  // (not a component of a closed partition)
  }
  return false;
}

// the context's error from a replay of component `comp`: verdict, event
// (as the component engine's key, for fill_stats) and the trace
void set_replay_event(tlcg_ctx* c, u64 comp, const CompReplay& rp) {
  c->status = rp.status;
  c->ev_level = rp.level;
  c->ev_comp = comp;
  c->ev_word = make_comp_event(rp.level, comp, 0, rp.action < 0 ? 15 : rp.action, rp.kind,
                               rp.invariant < 0 ? 0 : rp.invariant);
  c->ev_action = rp.action;
  c->ev_state = rp.trace.back();
  c->ev_parent_gidx = NO_PARENT;
  c->ev_parent_ref = NO_PARENT;
  c->xtrace_states = rp.trace;
  c->xtrace_acts = rp.acts;
  c->xtrace_valid = true;
}

// ---- component engine (component.h) ----

// device counters of a component pass (d_comp / h_comp)
constexpr int kCompCounters = 2 * COMP_MAXLV + 7;

// user invariants run only in the specialized kernels (jit.cpp: their device
// code is generated per model), so TLCG_JIT=0 leaves them to the global engine
bool jit_off() {
  const char* jv = std::getenv("TLCG_JIT");
  return jv && std::atoi(jv) == 0;
}

// applicable: `messages` immutable, one rank's components all local, local key fits 32 bits,
// N <= 8 (component_model.h packs N x N bit masks); user invariants need the specialized kernels
bool component_applicable(const tlcg_ctx* c) {
  const Layout& L = c->hm.L;
  const int mb = L.msg_sh + L.N * L.mw;
  return !L.producer && !c->opts.tlc_order && c->closed && L.bits <= 63 && L.bits - mb <= 32 && L.N <= 8 &&
         c->hm.n_init < (1ull << 36) && !(c->hm.user && jit_off());
}

// Fold the COMP_STRIPES copies of a pass's counters into out[0, kCompCounters)
// (the event and the overflow count live in copy 0 only) and reset every copy
// for the next pass, in stream order behind the pass: one small launch instead
// of two memsets before the pass and a 53-KB copy and a host fold after it
__global__ __launch_bounds__(128) void k_comp_finish(unsigned long long* __restrict__ ctr,
                                                     unsigned long long* __restrict__ out) {
  const int i = threadIdx.x;
  if (i >= kCompCounters) return;
  const bool single = i == COMP_MAXLV + 2 || i == COMP_MAXLV + 3;
  unsigned long long s = ctr[i];
  if (!single)
    for (int k = 1; k < COMP_STRIPES; ++k) s += ctr[(size_t)k * kCompCounters + i];
  out[i] = s;
  for (int k = 0; k < COMP_STRIPES; ++k) ctr[(size_t)k * kCompCounters + i] = k == 0 && i == COMP_MAXLV + 2 ? ~0ull : 0ull;
}

bool comp_scratch(tlcg_ctx* c, u64 n) {
  if (!c->d_comp) {
    // the copies, then the folded counters (k_comp_finish)
    const size_t bytes = sizeof(unsigned long long) * kCompCounters * (COMP_STRIPES + 1);
    if (!alloc_bytes(c, (void**)&c->d_comp, bytes, "component counters")) return false;
    HIPCHK(hipHostMalloc((void**)&c->h_comp, sizeof(unsigned long long) * kCompCounters));
    c->comp_clean = false;
  }
  if (n > c->ovf_cap) {
    hipFree(c->d_ovf[0]);
    hipFree(c->d_ovf[1]);
    c->d_ovf[0] = c->d_ovf[1] = nullptr;
    c->ovf_cap = 0;
    if (!alloc_bytes(c, (void**)&c->d_ovf[0], n * 8, "overflow list")) return false;
    if (!alloc_bytes(c, (void**)&c->d_ovf[1], n * 8, "overflow list")) return false;
    c->ovf_cap = n;
  }
  return true;
}

// Run every component of this rank on chip: K = 64, then the overflow at
// K = 128, then 255.  Returns 1 done, 0 some component does not fit (caller
// falls back to the global engine), -1 error.
int run_component(tlcg_ctx* c) {
  const HostModel& hm = c->hm;
  const Layout& L = hm.L;
  const int mb = L.msg_sh + L.N * L.mw;
  const u64 W = (u64)c->opts.world, R = (u64)c->opts.rank;
  const u64 r0 = c->range_hi ? 0 : hm.n_init * R / W;
  const u64 r1 = c->range_hi ? std::min<u64>(c->range_hi, hm.n_init) : hm.n_init * (R + 1) / W;
  c->engine = TLCG_ENGINE_COMPONENT;
  c->passes.clear();
  c->comp_levels.assign(COMP_MAXLV, 0);
  c->comp_level_gen.assign(COMP_MAXLV, 0);
  c->comp_init = r1 - r0;
  c->comp_generated = c->comp_distinct = c->comp_store_used = 0;
  c->outdeg.assign(3, 0);
  c->outdeg_valid = c->opts.outdegree;  // the component engine's parents are TLC's first discoverers
  c->pending = 0;
  if (!comp_scratch(c, std::max<u64>(r1 - r0, 1))) return -1;
  // specialize the kernels for these constants when the run is large enough
  // to repay a hipRTC compile (env TLCG_JIT=0/1 forces)
  const char* jv = std::getenv("TLCG_JIT");
  const bool want_jit = c->hm.user || (jv ? std::atoi(jv) != 0 : (r1 - r0) >= 65536);
  if (want_jit && c->jit_state == 0) {
    std::string e;
    c->jit_state = jit_build(L, c->opts.device, &c->jit, &e, c->user_src) ? 1 : -1;
    if (c->jit_state < 0) c->jit_error = e;
  }
  c->jit_used = want_jit && c->jit_state == 1;
  if (c->hm.user && !c->jit_used) return 0;  // (user invariants: the global engine, k_user_check)
  const char* cv = std::getenv("TLCG_CODE");  // 0: 32-bit local keys throughout (A/B)
  c->comp_code = code_bits(L) <= 16 && !(cv && std::atoi(cv) == 0);
  if (c->comp_code && !c->comp_mult) {
    const char* tv = std::getenv("TLCG_TUNE_MULT");  // 0: the default multiplier (A/B)
    c->comp_mult = tv && std::atoi(tv) == 0 ? DEFAULT_SLOT_MULT : tune_slot_mult(c->hm, CodeShape<64>::T, 1, 4096);  // (component_body.h)
  }
  // on-chip capacity cascade; the first step is tunable (TLCG_COMP_K0 = 32 / 64)
  int kCascade[4] = {64, 128, 255, 0};
  if (const char* k0 = std::getenv("TLCG_COMP_K0"))
    if (std::atoi(k0) == 32) {
      kCascade[0] = 32; kCascade[1] = 64; kCascade[2] = 128; kCascade[3] = 255;
    }
  u64 n = r1 - r0;
  int cur = -1;  // overflow list holding this pass's components (-1: range)
  u64 best_ev = NO_EVENT;
  for (int p = 0; p < 4 && kCascade[p] && n; ++p) {
    const int K = kCascade[p];
    const u64 base = c->comp_store_used;
    const u64 slots = component_store_slots(n, K);
    // the first pass runs component codes when they fit 16 bits (component_code.h);
    // a component whose initial key is no code, and the cascade, run 32-bit keys
    const bool code = p == 0 && K <= 64 && c->comp_code;
    tlcg_ctx::CompPass pass{K, base, r0, n, {}};
    // (its store holds records unless an A/B build of the specialized kernels asked for words)
    const char* jd = std::getenv("TLCG_JIT_DEFINES");
    pass.codes = code && !(c->jit_used && jd && std::strstr(jd, "TLCG_COMP_CODE_STORE=0"));
    if (pass.codes) {
      // 4 B per slot in the record buffer, none in the state store (16 B)
      if (c->crec_cap < slots) {
        hipFree(c->d_crec);
        c->d_crec = nullptr;
        c->crec_cap = 0;
        if (!alloc_bytes(c, (void**)&c->d_crec, slots * 4, "component records")) return -1;
        c->crec_cap = slots;
      }
    } else if (!ensure_store(c, base + slots)) {
      return -1;
    }
    if (cur >= 0) {
      pass.list.resize(n);
      HIPCHK_I(hipMemcpy(pass.list.data(), c->d_ovf[cur], n * 8, hipMemcpyDeviceToHost));
    }
    const int out = cur == 0 ? 1 : 0;
    if (!c->comp_clean) {  // (the first pass, or after a failed one; else k_comp_finish reset them)
      HIPCHK_I(hipMemsetAsync(c->d_comp, 0, sizeof(unsigned long long) * kCompCounters * COMP_STRIPES, c->stream));
      HIPCHK_I(hipMemsetAsync(c->d_comp + COMP_MAXLV + 2, 0xFF, sizeof(unsigned long long), c->stream));
    }
    c->comp_clean = false;
    CompArgs a;
    a.L = L;
    a.comp0 = r0;
    a.n_comp = n;
    a.list = cur >= 0 ? c->d_ovf[cur] : nullptr;
    if (pass.codes) {  // (the kernel writes records only; its word and parent pointers are not dereferenced)
      a.store = reinterpret_cast<u64*>(c->d_crec);
      a.parents = reinterpret_cast<u64*>(c->d_crec);
    } else {
      a.store = dev_state(c, base);
      a.parents = dev_parent(c, base);
    }
    a.store_base = base;
    a.msgs_bits = mb;
    a.rank_tag = (u64)c->opts.rank << 56;
    a.lvl = c->d_comp;
    a.totals = c->d_comp + COMP_MAXLV;
    a.event = c->d_comp + COMP_MAXLV + 2;
    a.ovf_n = c->d_comp + COMP_MAXLV + 3;
    a.outdeg = c->opts.outdegree ? c->d_comp + COMP_MAXLV + 4 : nullptr;
    a.lvl_gen = c->d_comp + COMP_MAXLV + 7;
    a.ovf_list = c->d_ovf[out];
    a.stripe = kCompCounters;
    a.nstripe = COMP_STRIPES;
    HIPCHK_I(hipEventRecord(c->e0, c->stream));
    // the code pass's slot hash, tuned on one component (all share its code graph)
    a.mult = code ? c->comp_mult : DEFAULT_SLOT_MULT;
    if (!(c->jit_used ? jit_launch_component(c->jit, a, K, code, c->stream) : launch_component(a, K, code, c->stream))) {
      c->err = "component kernel launch failed";
      return -1;
    }
    HIPCHK_I(hipEventRecord(c->e1, c->stream));
    unsigned long long* const folded = c->d_comp + (size_t)kCompCounters * COMP_STRIPES;
    k_comp_finish<<<1, 128, 0, c->stream>>>(c->d_comp, folded);
    HIPCHK_I(hipGetLastError());
    c->comp_clean = true;
    HIPCHK_I(hipMemcpyAsync(c->h_comp, folded, sizeof(unsigned long long) * kCompCounters, hipMemcpyDeviceToHost,
                            c->stream));
    HIPCHK_I(hipStreamSynchronize(c->stream));
    float ms = 0;
    hipEventElapsedTime(&ms, c->e0, c->e1);
    c->kernel_ms += ms;
    c->expand_ms += ms;
    for (int l = 0; l < COMP_MAXLV; ++l) {
      c->comp_levels[(size_t)l] += c->h_comp[l];
      c->comp_level_gen[(size_t)l] += c->h_comp[COMP_MAXLV + 7 + l];
    }
    c->comp_generated += c->h_comp[COMP_MAXLV];
    for (int i = 0; i < 3; ++i) c->outdeg[(size_t)i] += c->h_comp[COMP_MAXLV + 4 + i];
    c->comp_distinct += c->h_comp[COMP_MAXLV + 1];
    best_ev = std::min<u64>(best_ev, c->h_comp[COMP_MAXLV + 2]);
    c->comp_store_used = base + slots;
    if (pass.codes) c->win = base + slots;  // (the store's device window holds the passes after it)
    c->passes.push_back(std::move(pass));
    n = c->h_comp[COMP_MAXLV + 3];
    cur = out;
  }
  if (n) {  // components beyond 255 states / 48 levels: the global engine (or the tree) takes the model
    c->win = 0;
    c->passes.clear();
    return 0;
  }
  while (!c->comp_levels.empty() && c->comp_levels.back() == 0) c->comp_levels.pop_back();
  if (best_ev != NO_EVENT) {
    if (!resolve_comp_event(c, best_ev)) return -1;
    // like the level loop of the global engine, stop at the end of the level
    // that found the error: level E = the error's (the violating state's, or
    // the one after the failing / deadlocked state's) is complete, levels
    // 0..E-1 are expanded.  Lanes that found an error finished expanding their
    // level; the others ran their components out, so levels past E are cut.
    const size_t lv = (size_t)(best_ev >> 56) + 1;
    if (c->comp_levels.size() > lv) c->comp_levels.resize(lv);
    c->comp_distinct = 0;
    for (u64 x : c->comp_levels) c->comp_distinct += x;
    c->comp_generated = c->comp_init;  // initial states count as generated
    for (size_t l = 0; l + 1 < lv && l < c->comp_level_gen.size(); ++l) c->comp_generated += c->comp_level_gen[l];
    return 1;
  }
  c->status = TLCG_DONE;
  return 1;
}

// ---- component-tree engine (tree.h) ----

// applicable: Producer modelled (the component tree), one rank, one-word
// states, local keys < 32 bits, no TLC order (its lanes do not keep TLC's
// order), no outdegree statistics (they need TLC's first discoverers), no
// explicit device-store budget and no host FPSet tier (the tree keeps its
// whole store on the device: a run that must spill takes the global
// engine); TLCG_TREE=0 turns it off (A/B)
bool tree_applicable(const tlcg_ctx* c) {
  const Layout& L = c->hm.L;
  const int mb = L.msg_sh + L.N * L.mw;
  const char* tv = std::getenv("TLCG_TREE");
  return L.producer && !(tv && std::atoi(tv) == 0) && !c->no_tree && !c->opts.tlc_order && c->words == 1 &&
         L.bits - mb <= 31 && L.N >= 1 && L.N <= 8 && !c->opts.outdegree && L.nkv >= 1 && c->hm.n_init >= 1 &&
         !c->opts.device_store_cap && !c->opts.fpset_spill && !(c->hm.user && jit_off());
}

// the closed mode (tree.h): no Producer, a closed partition, components the
// component engine could not take (local keys over 32 bits, or more than 255
// states), codes of <= 31 bits (the LDS table stores code + 1)
bool tree_closed_applicable(const tlcg_ctx* c) {
  const Layout& L = c->hm.L;
  const char* tv = std::getenv("TLCG_TREE");
  return !L.producer && !(tv && std::atoi(tv) == 0) && c->closed && !c->opts.tlc_order && !c->opts.outdegree &&
         code_bits(L) <= 31 && L.N >= 1 && L.N <= 8 && (c->words == 1 || c->words == 2) &&
         c->hm.n_init >= 1 && c->hm.n_init < (1ull << 40) && !c->opts.device_store_cap && !c->opts.fpset_spill &&
         !(c->hm.user && (jit_off() || L.msgs_mask_hi));
}

// ---- the Producer tree's error, reported as TLC reports it ----
//
// TLC's queue order is the lexicographic order of each state's least
// shortest path from Init, as the sequence of Next ordinals it takes (a
// level is sorted by its states' first discoverers, which are sorted the
// same way).  The Producer's successors have the least ordinals
// (compaction.tla:216-219: its disjunct comes first, one ordinal per
// message), and BrokerCrash, the only other action enabled while
// `messages` is empty (CompactorPhaseOne needs Len(messages) > 0, :95),
// reads no message and commutes with it.  So every state whose
// `messages` starts with message m -- the component subtree m -- has a
// shortest path that produces m first, its least path starts with
// ordinal m, and TLC's queue holds every level >= 1 as subtree 0,
// subtree 1, .., then the states of the empty `messages` (the root).  The
// first error lies in the least subtree with an error at the least error
// level E, which the tree's kernel reports (tree_event_key); a TLC-order
// run of that subtree alone -- level 0 its seed state (message m produced
// from Init), levels up to E -- finds TLC's first error, its trace and its
// share of TLC's stop counters, and the tree's counts give the rest.  The
// subtree run's level sizes must equal the tree's depth histogram of the
// subtree (a state reached deeper than its depth would show at its own
// depth as a missing state), which checks the argument on the run itself;
// the subtrees before the erroring one (rarely any) are run to level E the
// same way.  Returns 1 reported, 0 the global engine must report it, -1 error.
void ensure_user_check(tlcg_ctx* c);

namespace {

// the tree's depth histogram of subtree m (levels 0..maxd), from the depth bytes of its chunks
bool subtree_depths(tlcg_ctx* c, u64 m, int maxd, std::vector<u64>* hist) {
  const Layout& L = c->hm.L;
  hist->assign((size_t)maxd + 1, 0);
  const u64 cap = (u64)c->tree_cap;
  u64 per = 1;  // components of subtree m in layer l: [m * per, (m + 1) * per), per = nkv^(l - 1)
  for (int l = 1; l <= L.N && (size_t)l < c->tree_layer_gbase.size(); ++l, per *= (u64)L.nkv) {
    const u64 c0 = m * per;
    std::vector<uint32_t> n(per);
    std::vector<uint8_t> dep(per * cap);
    HIPCHK(hipMemcpy(n.data(), c->d_tree_n + c->tree_layer_cbase[(size_t)l] + c0, per * 4, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(dep.data(), c->d_tree_dep + c->tree_layer_gbase[(size_t)l] + c0 * cap, per * cap,
                     hipMemcpyDeviceToHost));
    for (u64 i = 0; i < per; ++i)
      for (u64 k = 0; k < n[i] && k < cap; ++k)
        if (dep[i * cap + k] <= maxd) ++(*hist)[dep[i * cap + k]];
  }
  return true;
}

// a TLC-order run of subtree m to level E (absolute; its level r is level r + 1):
// the context, stopped on an error or after level E; nullptr on failure
// (TLCG_TIMING=1: the phases' wall times on stderr)
void phase_note(const char* what, double t0) {
  static const bool on = [] {
    const char* v = std::getenv("TLCG_TIMING");
    return v && std::atoi(v) != 0;
  }();
  if (on) std::fprintf(stderr, "[tlcg] %s %.3f ms\n", what, wall_ms() - t0);
}

tlcg_ctx* subtree_run(tlcg_ctx* c, u64 m, int E) {
  const Layout& L = c->hm.L;
  const double t0 = wall_ms();
  // sized from the tree's depth histogram of the subtree (its levels 1..E
  // are the run's; a larger run fails subtree_run_matches anyway), so the
  // FPSet and the store never regrow
  std::vector<u64> hist;
  if (!subtree_depths(c, m, E, &hist)) return nullptr;
  u64 n = 0;
  for (size_t l = 1; l < hist.size(); ++l) n += hist[l];
  if (c->sub && c->sub_cap < n + n / 8 + 4096) {  // (too small for this subtree: made again)
    tlcg_destroy(c->sub);
    c->sub = nullptr;
  }
  if (!c->sub) {
    tlcg_opts o = c->opts;
    o.world = 1;
    o.rank = 0;
    o.engine = TLCG_ENGINE_GLOBAL;
    o.tlc_order = 1;
    o.outdegree = 0;
    o.state_capacity = n + n / 4 + 4096;  // (headroom for the next error's subtree)
    int log2 = 16;
    while ((1ull << log2) < 2 * o.state_capacity && log2 < 40) ++log2;
    o.log2_fpset_slots = log2;
    o.fpset_spill = 0;
    o.device_store_cap = 0;
    tlcg_model md = c->model;
    if (tlcg_create(&md, &o, &c->sub) != 0) {
      tlcg_destroy(c->sub);
      c->sub = nullptr;
      return nullptr;
    }
    c->sub_cap = o.state_capacity;
    ensure_user_check(c);  // (one module for every subtree run of this context)
    if (c->ujit_state == 1) {
      c->sub->ujit = c->ujit;
      c->sub->ujit_state = 2;
    }
  }
  tlcg_ctx* t = c->sub;
  phase_note("subtree create", t0);
  t->seed_valid = true;
  t->seed_state = producer_succ<u64>(L, init_state<u64>(L, 0), 0, (int)m);
  tlcg_stats st;
  if (tlcg_init(t, &st) != 0) return nullptr;
  while (t->status == TLCG_RUNNING && (int)t->level_base.size() - 1 < E)
    if (tlcg_step_level(t, &st) != 0) return nullptr;
  phase_note("subtree run", t0);
  return t;
}

// the run's level sizes (relative levels 0..k) against the tree's depths 1..k + 1 of the subtree
bool subtree_run_matches(tlcg_ctx* c, tlcg_ctx* t, u64 m, int E) {
  std::vector<u64> hist;
  if (!subtree_depths(c, m, E, &hist)) return false;
  for (int r = 0; r + 1 <= E; ++r) {
    const u64 got = (size_t)r + 1 < t->level_base.size() ? t->level_base[(size_t)r + 1] - t->level_base[(size_t)r] : 0;
    if (got != hist[(size_t)r + 1]) return false;
  }
  return true;
}

int producer_error(tlcg_ctx* c, u64 evk) {
  const Layout& L = c->hm.L;
  const int E = (int)(evk >> 40);
  const u64 sub = evk & ((1ull << 40) - 1);
  if (E < 2 || sub >= (u64)L.nkv || sub > 8 || c->words != 1 || c->hm.n_init != 1) return 0;
  // the subtrees before: no error up to level E (sub is the least with one); their levels E - 1, E
  u64 pre_lm1 = 0, pre_l = 0, pre_gen = 0;
  for (u64 m = 0; m < sub; ++m) {
    tlcg_ctx* t = subtree_run(c, m, E);
    if (!t) return 0;
    const bool ok = t->status == TLCG_RUNNING || t->status == TLCG_DONE;
    std::vector<u64> lg(4096);
    int32_t ng = 0;
    const bool good = ok && subtree_run_matches(c, t, m, E) && tlcg_level_generated(t, lg.data(), 4096, &ng) == 0;
    if (good) {
      auto lv = [&](int r) -> u64 {
        return (size_t)r + 1 < t->level_base.size() ? t->level_base[(size_t)r + 1] - t->level_base[(size_t)r] : 0;
      };
      pre_lm1 += lv(E - 2);
      pre_l += lv(E - 1);
      pre_gen += E - 1 < ng ? lg[(size_t)E - 1] : 0;  // (lg[k]: generated by expanding relative level k - 1)
    }
    if (!good) return 0;
  }
  const double t0 = wall_ms();
  tlcg_ctx* t = subtree_run(c, sub, E);
  if (!t) return 0;
  int res = 0;
  uint64_t g = 0, d = 0, q = 0;
  std::vector<uint64_t> tst(4096);
  std::vector<int32_t> tact(4096);
  int32_t tn = 0;
  tlcg_stats ts;
  if (t->status >= TLCG_VIOLATION && t->ev_level == E - 1 && subtree_run_matches(c, t, sub, E) &&
      tlcg_tlc_stop_stats(t, &g, &d, &q) == 0 && tlcg_trace_words(t, tst.data(), tact.data(), 4096, &tn) == 0 &&
      tn >= 1 && tn < 4096) {
    fill_stats(t, &ts);
    auto lv = [&](int r) -> u64 {
      return (size_t)r + 1 < t->level_base.size() ? t->level_base[(size_t)r + 1] - t->level_base[(size_t)r] : 0;
    };
    // the subtree run's share at its stop (p: the stopping state, relative level E - 2)
    u64 below = 0, upto = 0;  // its states in levels < E - 2, <= E - 2
    for (int r = 0; r < E - 1; ++r) (r < E - 2 ? below : upto) += lv(r);
    upto += below;
    const u64 within = g - t->gen_at[(size_t)E - 2];   // level E - 2's out-degrees before p, and p's counted ones
    const u64 found = d - upto;                         // level E - 1 states found by the stop
    const u64 rank = (d - q - 1) - below;               // p's place in its level
    // the whole model: the tree's full levels, the subtrees before, the share
    auto at = [](const std::vector<u64>& v, int i) -> u64 { return i >= 0 && (size_t)i < v.size() ? v[(size_t)i] : 0; };
    u64 gen = c->comp_init, dist = 0, pos = 0;
    for (int l = 0; l < E - 1; ++l) {
      gen += at(c->comp_level_gen, l);
      pos += at(c->comp_levels, l);
    }
    for (int l = 0; l <= E - 1; ++l) dist += at(c->comp_levels, l);
    c->stop_g = gen + pre_gen + within;
    c->stop_d = dist + pre_l + found;
    c->stop_q = c->stop_d - (pos + pre_lm1 + rank + 1);
    c->stop_cached = true;
    // the verdict and TLC's trace: Init, the Producer's step to the seed, the subtree run's
    c->status = t->status;
    c->ev_level = E;
    const int kind = t->status == TLCG_VIOLATION ? EVK_VIOLATION : t->status == TLCG_INVARIANT_ERROR ? EVK_INV_ERROR
                   : t->status == TLCG_DEADLOCK ? EVK_DEADLOCK : EVK_ACTION_ERROR;
    c->ev_word = make_comp_event(E, sub, 0, ts.action < 0 ? 15 : ts.action, kind, ts.invariant < 0 ? 0 : ts.invariant);
    c->ev_action = ts.action;
    c->ev_parent_gidx = NO_PARENT;
    c->ev_parent_ref = NO_PARENT;
    c->xtrace_states.assign(1, (u128)init_state<u64>(L, 0));
    c->xtrace_acts.assign(1, TLCG_ACT_INIT);
    for (int i = 0; i < tn; ++i) {
      c->xtrace_states.push_back((u128)tst[(size_t)i]);
      c->xtrace_acts.push_back(i == 0 ? (int)ACT_PRODUCER : tact[(size_t)i]);
    }
    c->ev_state = c->xtrace_states.back();
    c->xtrace_valid = true;
    // the counts at the end of level E, as every engine reports them
    if (c->comp_levels.size() > (size_t)E + 1) c->comp_levels.resize((size_t)E + 1);
    c->comp_distinct = 0;
    for (u64 x : c->comp_levels) c->comp_distinct += x;
    c->comp_generated = c->comp_init;
    for (size_t l = 0; l < (size_t)E && l < c->comp_level_gen.size(); ++l) c->comp_generated += c->comp_level_gen[l];
    c->kernel_ms += t->kernel_ms;
    c->expand_ms += t->expand_ms;
    res = 1;
  }
  phase_note("subtree report", t0);
  return res;
}

}  // namespace

// Run the component tree.  Producer modelled: every layer, chunks of 384
// states per component (the shipped N = 3, C = 3, K = 1 have at most 359),
// then 1024 if one overflows.  Closed: this rank's components (a contiguous
// range of initial states) in one launch, chunks of 640 states (557 at
// CompactionTimesLimit = 12), then 2048.  Returns 1 done, 0 the global engine
// takes the model (an event to report as TLC does, a component past the
// capacity or TREE_MAXLV depths, or not enough memory), -1 error.
int run_tree(tlcg_ctx* c) {
  const Layout& L = c->hm.L;
  const bool closed = !L.producer;
  std::vector<u64> ncomp;  // components per launch (layer): nkv^l, or this rank's initial states
  std::vector<u64> lbase;  // the layer's number of the launch's component 0
  u64 r0 = 0;
  const u64 W = (u64)c->opts.world, R = (u64)c->opts.rank;
  int shard = 0;  // Producer, W > 1: the layer whose components are split between the ranks
  if (closed) {
    r0 = c->range_hi ? 0 : c->hm.n_init * R / W;
    ncomp.push_back(c->range_hi ? std::min<u64>(c->range_hi, c->hm.n_init) : c->hm.n_init * (R + 1) / W - r0);
    lbase.push_back(0);
  } else {
    // every component of layer l >= 1 lies in the subtree of one component of
    // layer `shard` (its first `shard` messages; compaction.tla:83-87 only
    // appends), so the ranks split layer `shard` into contiguous ranges and
    // each runs its subtrees alone -- no exchange.  The layers above it (a
    // few components) run on every rank and count on rank 0.
    u64 width = 1;
    if (W > 1)
      while (shard < L.N && width < W) {
        width *= (u64)L.nkv;
        ++shard;
      }
    const u64 a = width * R / W, b = width * (R + 1) / W;
    u64 full = 1;  // nkv^l
    for (int l = 0; l <= L.N; ++l) {
      if (l) {
        if (full > (1ull << 34) / (u64)L.nkv) return 0;
        full *= (u64)L.nkv;
      }
      if (W == 1 || l < shard) {
        ncomp.push_back(full);
        lbase.push_back(0);
      } else {
        const u64 per = full / width;  // nkv^(l - shard)
        ncomp.push_back((b - a) * per);
        lbase.push_back(a * per);
      }
    }
  }
  u64 comps = 0;
  for (u64 x : ncomp) comps += x;
  if (!c->d_tree_ctr) {
    const size_t bytes = sizeof(unsigned long long) * (2 * TREE_MAXLV * TREE_STRIPES + 3);
    if (!alloc_bytes(c, (void**)&c->d_tree_ctr, bytes, "tree counters")) return -1;
    HIPCHK_I(hipHostMalloc((void**)&c->h_tree_ctr, bytes));
  }
  // components per wavefront (tuning hook TLCG_TREE_G = 1 / 2 / 4)
  int groups = 4;
  if (const char* gv = std::getenv("TLCG_TREE_G")) groups = std::atoi(gv) == 1 ? 1 : std::atoi(gv) == 2 ? 2 : 4;
  if (closed && groups == 1) groups = 2;
  // the layout-specialized kernels (jit.cpp) when the tree is large enough
  // to repay a hipRTC compile (env TLCG_JIT=0/1 forces)
  const char* jv = std::getenv("TLCG_JIT");
  const bool want_jit = (c->hm.user || (jv ? std::atoi(jv) != 0 : comps >= 4096)) && groups == 4;
  if (want_jit && c->jit_state == 0) {
    std::string e;
    c->jit_state = jit_build(L, c->opts.device, &c->jit, &e, c->user_src) ? 1 : -1;
    if (c->jit_state < 0) c->jit_error = e;
  }
  c->jit_used = want_jit && c->jit_state == 1;
  if (c->hm.user && !c->jit_used) return 0;  // (user invariants: the global engine, k_user_check)
  const int words = c->words;
  if (closed && !c->tree_mult) {  // (640-slot tables, 16 lanes per component; tree_body.h)
    const char* tv = std::getenv("TLCG_TUNE_MULT");
    c->tree_mult = tv && std::atoi(tv) == 0 ? DEFAULT_SLOT_MULT : tune_slot_mult(c->hm, 640, 16, 4096);
    // (zero displacements when none is found: the plain multiply-shift slot)
    build_slot_disp(c->hm, 640, c->tree_mult, &c->tree_disp_mult, c->tree_disp);
  }
  for (int cap : closed ? std::vector<int>{640, 2048} : std::vector<int>{384, 1024}) {
    const u64 slots = comps * (u64)cap;
    // the store (state words + parent), the depth bytes and the sizes must fit next to what is allocated
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) != hipSuccess) return 0;
    const double per_slot = 8.0 * (words + 1) + (closed ? 0.0 : 1.0);
    const double have = (double)fr + 8.0 * (words + 1) * (double)c->cap + (double)c->tree_slots + 4.0 * (double)c->tree_comps;
    if (per_slot * (double)slots + 4.0 * (double)comps > 0.85 * have) return 0;
    c->engine = TLCG_ENGINE_TREE;
    c->comp_store_used = 0;  // nothing of an earlier run to keep (tlcg_init freed the host chunks)
    if (!ensure_store(c, slots)) return -1;
    if (!closed && c->tree_slots < slots) {
      hipFree(c->d_tree_dep);
      c->d_tree_dep = nullptr;
      c->tree_slots = 0;
      if (!alloc_bytes(c, (void**)&c->d_tree_dep, slots, "tree depths")) return -1;
      c->tree_slots = slots;
    }
    if (c->tree_comps < comps) {
      hipFree(c->d_tree_n);
      c->d_tree_n = nullptr;
      c->tree_comps = 0;
      if (!alloc_bytes(c, (void**)&c->d_tree_n, comps * 4, "tree sizes")) return -1;
      c->tree_comps = comps;
    }
    unsigned long long* ctr = c->d_tree_ctr;
    constexpr int kTreeCtr = 2 * TREE_MAXLV * TREE_STRIPES + 3;  // [stripe][lvl, lvl_gen], flags, max_n, event
    HIPCHK_I(hipMemsetAsync(ctr, 0, sizeof(unsigned long long) * (kTreeCtr - 1), c->stream));
    HIPCHK_I(hipMemsetAsync(ctr + kTreeCtr - 1, 0xFF, sizeof(unsigned long long), c->stream));
    HIPCHK_I(hipEventRecord(c->e0, c->stream));
    u64 gbase = 0, cbase = 0, pgbase = 0, pcbase = 0;
    c->tree_layer_gbase.clear();
    c->tree_layer_cbase.clear();
    for (size_t l = 0; l < ncomp.size(); ++l) {
      c->tree_layer_gbase.push_back(gbase);
      c->tree_layer_cbase.push_back(cbase);
      TreeArgs a;
      a.L = L;
      a.layer = (int)l;
      a.n_comp = ncomp[l];
      a.n_init = c->hm.n_init;
      a.comp0 = r0;
      a.comp_base = lbase[l];
      a.par_comp_base = l ? lbase[l - 1] : 0;
      a.count = closed || W == 1 || (int)l >= shard || R == 0;
      a.par_states = l ? c->d_states + pgbase : nullptr;
      a.par_dep = l ? c->d_tree_dep + pgbase : nullptr;
      a.par_n = l ? c->d_tree_n + pcbase : nullptr;
      a.par_gbase = pgbase;
      a.states = c->d_states + gbase * (u64)words;
      a.parents = c->d_parents + gbase;
      a.dep = closed ? nullptr : c->d_tree_dep + gbase;
      a.n_out = c->d_tree_n + cbase;
      a.gbase = gbase;
      a.rank_tag = (u64)c->opts.rank << 56;
      a.lvl = ctr;
      a.lvl_gen = ctr + TREE_MAXLV;
      a.flags = reinterpret_cast<unsigned int*>(ctr + 2 * TREE_MAXLV * TREE_STRIPES);
      a.max_n = reinterpret_cast<unsigned int*>(ctr + 2 * TREE_MAXLV * TREE_STRIPES + 1);
      a.event = ctr + kTreeCtr - 1;
      a.stripe = 2 * TREE_MAXLV;
      a.nstripe = TREE_STRIPES;
      a.mult = closed ? c->tree_mult : DEFAULT_SLOT_MULT;
      a.disp_mult = c->tree_disp_mult;
      std::copy(c->tree_disp, c->tree_disp + TREE_DISP, a.disp);  // (zeros unless closed)
      const bool jit = c->jit_used && (cap == 384 || cap == 1024 || cap == 640 || cap == 2048);
      const int g = cap == 384 || cap == 640 ? groups : 1;
      if (!(jit ? jit_launch_tree(c->jit, a, cap, c->stream) : launch_tree(a, cap, g, closed, words, c->stream))) {
        c->err = "component-tree kernel launch failed";
        return -1;
      }
      pgbase = gbase;
      pcbase = cbase;
      gbase += a.n_comp * (u64)cap;
      cbase += a.n_comp;
    }
    HIPCHK_I(hipEventRecord(c->e1, c->stream));
    HIPCHK_I(hipMemcpyAsync(c->h_tree_ctr, ctr, sizeof(unsigned long long) * kTreeCtr, hipMemcpyDeviceToHost,
                            c->stream));
    HIPCHK_I(hipStreamSynchronize(c->stream));
    for (int sidx = 1; sidx < TREE_STRIPES; ++sidx)  // fold the stripes into copy 0
      for (int i = 0; i < 2 * TREE_MAXLV; ++i) c->h_tree_ctr[i] += c->h_tree_ctr[(size_t)sidx * 2 * TREE_MAXLV + i];
    float ms = 0;
    hipEventElapsedTime(&ms, c->e0, c->e1);
    c->kernel_ms += ms;
    c->expand_ms += ms;
    const unsigned flags = (unsigned)c->h_tree_ctr[2 * TREE_MAXLV * TREE_STRIPES];
    if (flags & TREE_EVENT) {  // (Producer modelled) the global engine finds TLC's first error and its trace
      c->tree_event = true;
      return 0;
    }
    if (flags & TREE_OVERFLOW) continue;
    const u64 evk = c->h_tree_ctr[kTreeCtr - 1];  // closed mode: the least error key (tree_event_key)
    c->tree_cap = cap;
    // (the closed mode's store holds codes unless an A/B build asked for words)
    const char* jd = std::getenv("TLCG_JIT_DEFINES");
    c->tree_codes = closed && !(jd && std::strstr(jd, "TLCG_TREE_CODE_STORE=0"));
    c->tree_r0 = r0;
    if (std::getenv("TLCG_TREE_STATS")) {  // diagnostics: component sizes per layer
      std::vector<uint32_t> nn(comps);
      HIPCHK_I(hipMemcpy(nn.data(), c->d_tree_n, comps * 4, hipMemcpyDeviceToHost));
      u64 b0 = 0;
      for (size_t l = 0; l < ncomp.size(); ++l) {
        uint32_t mx = 0, mn = ~0u;
        double sum = 0;
        for (u64 i = 0; i < ncomp[l]; ++i) {
          mx = std::max(mx, nn[b0 + i]);
          mn = std::min(mn, nn[b0 + i]);
          sum += nn[b0 + i];
        }
        std::fprintf(stderr, "tree layer %zu: %llu components, states min %u avg %.1f max %u\n", l,
                     (unsigned long long)ncomp[l], mn, sum / (double)ncomp[l], mx);
        b0 += ncomp[l];
      }
    }
    c->passes.clear();
    c->comp_levels.assign(c->h_tree_ctr, c->h_tree_ctr + TREE_MAXLV);
    c->comp_level_gen.assign(c->h_tree_ctr + TREE_MAXLV, c->h_tree_ctr + 2 * TREE_MAXLV);
    while (!c->comp_levels.empty() && c->comp_levels.back() == 0) c->comp_levels.pop_back();
    c->comp_init = closed ? ncomp[0] : R == 0 ? c->hm.n_init : 0;  // (Init counts once, on rank 0)
    c->comp_distinct = 0;
    for (u64 x : c->comp_levels) c->comp_distinct += x;
    c->comp_generated = c->comp_init;
    for (u64 x : c->comp_level_gen) c->comp_generated += x;
    c->comp_store_used = slots;
    c->outdeg_valid = false;
    c->pending = 0;
    c->status = TLCG_DONE;
    if (closed && evk != ~0ull) {
      // TLC's first error: the least component with an error at the least
      // level, replayed on the host in TLC's order (trace, event); the counts
      // are those at the end of level E, as every engine reports them
      const int E = (int)(evk >> 40);
      const u64 comp = evk & ((1ull << 40) - 1);
      CompReplay rp;
      if (!replay_component(c, comp, &rp) || rp.level != E) {
        c->err = "internal: the component tree's error was not found by its replay";
        return -1;
      }
      set_replay_event(c, comp, rp);
      if (c->comp_levels.size() > (size_t)E + 1) c->comp_levels.resize((size_t)E + 1);
      c->comp_distinct = 0;
      for (u64 x : c->comp_levels) c->comp_distinct += x;
      c->comp_generated = c->comp_init;
      for (size_t l = 0; l < (size_t)E && l < c->comp_level_gen.size(); ++l) c->comp_generated += c->comp_level_gen[l];
    } else if (!closed && evk != ~0ull) {
      // Producer modelled: TLC's first error from the one subtree holding it
      // (producer_error); else (several ranks, an error of the root
      // component or at level 0 / 1, a check failed) the global engine
      // reports it, in TLC order on one rank
      const int pr = W == 1 ? producer_error(c, evk) : 0;
      if (pr < 0) return -1;
      if (pr == 0) {
        c->tree_event = true;
        return 0;
      }
    }
    return 1;
  }
  return 0;  // a component past the largest chunk
}

// the global engine's user-check module (jit.h JitUserCheck), built once per
// context (hipRTC; cached on disk after the first build)
void ensure_user_check(tlcg_ctx* c) {
  if (c->ujit_state != 0 || !c->hm.user) return;
  std::string e;
  c->ujit_state = !jit_off() && jit_build_user_check(c->hm.L, c->opts.device, c->user_src, &c->ujit, &e) ? 1 : -1;
  if (c->ujit_state < 0 && !jit_off()) c->jit_error = e;
}

// the least user-invariant event of the new level [g0, g0 + n) (NO_EVENT: none,
// or no user invariants); ~0ull - 1 on a launch error
u64 user_check_level(tlcg_ctx* c, u64 g0, u64 n, bool level0) {
  if (!c->hm.user || !n) return NO_EVENT;
  unsigned long long h = NO_EVENT;
  if (hipMemcpyAsync(c->d_uev, &h, sizeof h, hipMemcpyHostToDevice, c->stream) != hipSuccess) return ~0ull - 1;
  const UserCheckArgs a = {dev_state(c, g0), dev_parent(c, g0), n, level0 ? 1 : 0, c->d_uev,
                           (u64)c->opts.rank << 56, g0};
  ensure_user_check(c);
  if (c->ujit_state >= 1) {
    if (!jit_launch_user_check(c->ujit, a, c->stream)) {
      c->err = "user-invariant check launch failed";
      return ~0ull - 1;
    }
  } else {
    const unsigned g = grid_for(n, BLOCK, 0x7fffffffu);
    if (c->words == 1)
      k_user_check<u64><<<g, BLOCK, 0, c->stream>>>(c->hm.L, c->d_prog, a);
    else
      k_user_check<u128><<<g, BLOCK, 0, c->stream>>>(c->hm.L, c->d_prog, a);
  }
  if (hipGetLastError() != hipSuccess ||
      hipMemcpyAsync(&h, c->d_uev, sizeof h, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
      hipStreamSynchronize(c->stream) != hipSuccess) {
    c->err = "user-invariant check failed";
    return ~0ull - 1;
  }
  return h;
}

bool run_init(tlcg_ctx* c) {
  c->engine = TLCG_ENGINE_GLOBAL;
  const HostModel& hm = c->hm;
  const Layout& L = hm.L;
  c->level_base.assign(1, 0);
  c->gen_at.clear();
  c->outdeg.assign(1, 0);
  c->outdeg_valid = c->opts.outdegree && c->opts.tlc_order && c->opts.world == 1;
  c->generated = 0;
  c->status = TLCG_RUNNING;
  c->ev_word = NO_EVENT;
  c->ev_level = -1;
  c->ev_parent_gidx = NO_PARENT;
  c->ev_parent_ref = NO_PARENT;
  c->ev_action = -1;
  c->kernel_ms = c->expand_ms = 0;
  c->levels_redone = 0;
  const int world = c->opts.world;
  if (c->seed_valid) {  // level 0 = the one seed state (producer_error), one rank
    if (!ensure_store(c, 1)) return false;
    if (!rebuild_fpset(c, c->d_slots ? c->log2 : 16, 0)) return false;
    uint64_t w[2] = {0, 0}, par = NO_PARENT;
    split_words(c->seed_state, w, c->words);
    HIPCHK(hipMemcpy(dev_state(c, 0), w, 8 * (size_t)c->words, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(dev_parent(c, 0), &par, 8, hipMemcpyHostToDevice));
    if (!rebuild_fpset(c, c->log2, 1)) return false;  // (inserts it)
    c->generated = 1;
    c->level_base.push_back(1);
    return true;
  }
  u64 expect = world == 1 ? hm.n_init : hm.n_init / (u64)world + hm.n_init / (u64)(4 * world) + 4096;
  expect = std::min(expect, hm.n_init);
  if (!ensure_store(c, expect)) return false;
  if (!c->d_slots) {
    int l = c->opts.log2_fpset_slots > 0 ? c->opts.log2_fpset_slots : c->opts.fpset_spill ? 10 : 16;
    while ((1ull << l) < 2 * expect && c->opts.log2_fpset_slots <= 0 && l < 40) ++l;
    if (!rebuild_fpset(c, l, 0)) return false;
  } else {
    if (!rebuild_fpset(c, c->log2, 0)) return false;  // clear
    if (!ensure_fpset(c, expect)) return false;
  }
  for (;;) {
    if (!reset_ctr(c)) return false;
    HIPCHK_I(hipEventRecord(c->e0, c->stream));
    const unsigned g = grid_for(hm.n_init, BLOCK, 0x7fffffffu);
    if (world == 1 && c->words == 1) {
      k_init_direct<u64><<<g, BLOCK, 0, c->stream>>>(L, hm.n_init, c->d_slots, c->log2, c->d_states, c->d_parents,
                                                     c->d_ctr);
    } else if (world == 1) {
      k_init_direct<u128><<<g, BLOCK, 0, c->stream>>>(L, hm.n_init, c->d_slots, c->log2, (u128*)c->d_states,
                                                      c->d_parents, c->d_ctr);
    } else if (c->words == 1) {
      k_init_part<u64><<<g, BLOCK, 0, c->stream>>>(L, hm.n_init, c->opts.rank, world, c->owner_mask, c->d_slots,
                                                   c->log2, c->d_states, c->d_parents, c->cap, c->d_ctr);
    } else {
      k_init_part<u128><<<g, BLOCK, 0, c->stream>>>(L, hm.n_init, c->opts.rank, world, c->owner_mask, c->d_slots,
                                                    c->log2, (u128*)c->d_states, c->d_parents, c->cap, c->d_ctr);
    }
    HIPCHK_I(hipGetLastError());
    HIPCHK_I(hipEventRecord(c->e1, c->stream));
    if (!read_ctr(c)) return false;
    float ms = 0;
    hipEventElapsedTime(&ms, c->e0, c->e1);
    c->kernel_ms += ms;
    const unsigned ovf = c->h_ctr->overflow;
    if (ovf & OVF_DUP_INIT) {
      c->err = "internal: duplicate initial state";
      return false;
    }
    if (ovf & OVF_WIDE_SPIN) {
      c->err = "internal: wide FPSet slot never published";
      return false;
    }
    if (!ovf) break;
    ++c->levels_redone;
    if (ovf & OVF_STORE) {
      if (!ensure_store(c, std::max<u64>(c->h_ctr->n_new, c->cap * 2))) return false;
    }
    if (!rebuild_fpset(c, c->log2 + ((ovf & OVF_FPSET) ? 1 : 0), 0)) return false;
  }
  const u64 n_new = world == 1 ? hm.n_init : c->h_ctr->n_new;
  c->generated = n_new;
  // partitioned ranks keep every level (possibly empty) so that level d is
  // the same BFS level on every rank; termination is decided globally.
  if (n_new || world > 1) c->level_base.push_back(n_new);
  const u64 uev = user_check_level(c, 0, n_new, true);
  if (uev == ~0ull - 1) return false;
  const u64 ev = std::min<u64>(c->h_ctr->event, uev);
  if (ev != NO_EVENT) return resolve_event(c, ev, 0);
  if (!n_new && world == 1) c->status = TLCG_DONE;
  return true;
}

template <bool P, bool T, bool X>
void launch_expand_t(const ExpandArgs& a, unsigned grid, hipStream_t s, int words) {
  if (words == 1) k_expand<u64, P, T, X><<<grid, BLOCK, 0, s>>>(a);
  else if constexpr (!X) k_expand<u128, P, T, false><<<grid, BLOCK, 0, s>>>(a);  // wide: closed partitions only
}

bool launch_expand(tlcg_ctx* c, u64 front0, u64 n_front, bool part) {
  const Layout& L = c->hm.L;
  ExpandArgs a;
  a.L = L;
  a.frontier = dev_state(c, front0);
  a.n_front = n_front;
  a.front_gidx0 = front0;
  a.slots = c->d_slots;
  a.log2 = c->log2;
  const u64 d = distinct_of(c);
  a.states_out = dev_state(c, d);
  a.parents_out = dev_parent(c, d);
  a.cap_out = dev_room(c, d);
  a.slot_out = c->d_slot_new;
  a.dkey_slot = c->d_dkey_slot;
  a.ctr = c->d_ctr;
  a.rank_tag = (u64)c->opts.rank << 56;
  a.rank = c->opts.rank;
  a.world = c->opts.world;
  a.owner_mask = c->owner_mask;
  a.outbox = c->d_outbox;
  a.outbox_cap = c->outbox_cap;
  const bool prod = L.producer != 0, tlc = c->opts.tlc_order != 0;
  if (!prod && !tlc && !part && c->fast_items > 0 && c->words == 1) {
    const int it = c->fast_items;
    const unsigned g = grid_for(n_front, (u64)BLOCK * it, c->grid_cap);
    if (c->probe_mode == 0) {
      if (it == 1) k_expand_fast<1, 0><<<g, BLOCK, 0, c->stream>>>(a);
      else if (it == 2) k_expand_fast<2, 0><<<g, BLOCK, 0, c->stream>>>(a);
      else k_expand_fast<4, 0><<<g, BLOCK, 0, c->stream>>>(a);
    } else {
      if (it == 1) k_expand_fast<1, 1><<<g, BLOCK, 0, c->stream>>>(a);
      else if (it == 2) k_expand_fast<2, 1><<<g, BLOCK, 0, c->stream>>>(a);
      else k_expand_fast<4, 1><<<g, BLOCK, 0, c->stream>>>(a);
    }
    HIPCHK_I(hipGetLastError());
    return true;
  }
  if (prod && !tlc && !part && c->fast_items > 0 && c->words == 1) {
    k_expand_prod<8><<<grid_for(n_front, 2 * BLOCK, c->grid_cap), BLOCK, 0, c->stream>>>(a);
    HIPCHK_I(hipGetLastError());
    return true;
  }
  const u64 per_block = (u64)BLOCK * (prod ? 1 : ITEMS);
  const unsigned grid = grid_for(n_front, per_block, c->grid_cap);
  const int w = c->words;
  if (prod) {
    if (tlc) launch_expand_t<true, true, false>(a, grid, c->stream, w);
    else if (part) launch_expand_t<true, false, true>(a, grid, c->stream, w);
    else launch_expand_t<true, false, false>(a, grid, c->stream, w);
  } else {
    if (tlc) launch_expand_t<false, true, false>(a, grid, c->stream, w);
    else if (part) launch_expand_t<false, false, true>(a, grid, c->stream, w);
    else launch_expand_t<false, false, false>(a, grid, c->stream, w);
  }
  HIPCHK_I(hipGetLastError());
  return true;
}

// TLC -workers 1 order for the level just expanded: sort the new states by
// their first-discovery key (parent position, successor ordinal).
bool tlc_order_level(tlcg_ctx* c, u64 n_new) {
  if (!n_new) return true;
  const Layout& L = c->hm.L;
  const u64 d = distinct_of(c);
  k_gather_dkey<<<grid_for(n_new, BLOCK, 0x7fffffffu), BLOCK, 0, c->stream>>>(n_new, c->d_slot_new,
                                                                              c->d_dkey_slot, c->d_dk);
  HIPCHK_I(hipGetLastError());
  const int end_bit = std::min(64, bits_for(((d + n_new) << L.ord_bits) | ((1ull << L.ord_bits) - 1)));
  size_t tmp = c->sort_tmp_bytes;
  const unsigned g = grid_for(n_new, BLOCK, 0x7fffffffu);
  const u64 tag = (u64)c->opts.rank << 56;
  if (c->words == 1) {
    HIPCHK_I(hipcub::DeviceRadixSort::SortPairs(c->d_sort_tmp, tmp, c->d_dk, c->d_dk2, dev_state(c, d), c->d_st2,
                                                (int)n_new, 0, end_bit, c->stream));
    k_tlc_finish<u64><<<g, BLOCK, 0, c->stream>>>(L, n_new, c->d_st2, c->d_dk2, dev_state(c, d), dev_parent(c, d),
                                                  tag, c->d_ctr);
  } else {
    u128* st = (u128*)dev_state(c, d);
    HIPCHK_I(hipcub::DeviceRadixSort::SortPairs(c->d_sort_tmp, tmp, c->d_dk, c->d_dk2, (const u128*)st,
                                                (u128*)c->d_st2, (int)n_new, 0, end_bit, c->stream));
    k_tlc_finish<u128><<<g, BLOCK, 0, c->stream>>>(L, n_new, (const u128*)c->d_st2, c->d_dk2, st, dev_parent(c, d),
                                                   tag, c->d_ctr);
  }
  HIPCHK_I(hipGetLastError());
  return true;
}

// expected new states of the next level: the last level's growth ratio (with
// headroom), capped by the per-state bound
u64 next_level_estimate(const tlcg_ctx* c, u64 F) {
  const HostModel& hm = c->hm;
  const size_t n = c->level_base.size();
  double ratio = 2.0;
  if (n >= 3) {
    const u64 prev = c->level_base[n - 2] - c->level_base[n - 3];
    if (prev) ratio = std::max(ratio, 1.5 * (double)F / (double)prev);
  }
  ratio = std::min(ratio, (double)hm.max_new_per_state);
  return (u64)(ratio * (double)F) + 1024;
}

// TLC's outdegree histogram from a finished TLC-order level: runs of equal
// parent in the new level [d, d + n_new), the F - runs parents without one
bool add_child_runs(tlcg_ctx* c, u64 d, u64 n_new, u64 F) {
  std::vector<unsigned long long> h(OUTDEG_BINS, 0);
  if (n_new) {
    if (!c->d_runs && !alloc_bytes(c, (void**)&c->d_runs, OUTDEG_BINS * 8, "outdegree histogram")) return false;
    HIPCHK(hipMemsetAsync(c->d_runs, 0, OUTDEG_BINS * 8, c->stream));
    // the level sits in the device window unless a spill moved it (then it is
    // the frontier of the next step, still on the device)
    k_child_runs<<<grid_for(n_new, BLOCK, 0x7fffffffu), BLOCK, 0, c->stream>>>(dev_parent(c, d), n_new,
                                                                              c->hm.L.ord_bits, c->d_runs);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(h.data(), c->d_runs, OUTDEG_BINS * 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
  }
  u64 runs = 0;
  for (int k = 1; k < OUTDEG_BINS; ++k) runs += h[(size_t)k];
  h[0] = F - runs;
  if (c->outdeg.size() < (size_t)OUTDEG_BINS) c->outdeg.resize(OUTDEG_BINS, 0);
  for (int k = 0; k < OUTDEG_BINS; ++k) c->outdeg[(size_t)k] += h[(size_t)k];
  return true;
}

bool step_level(tlcg_ctx* c) {
  if (c->status != TLCG_RUNNING) return true;
  const HostModel& hm = c->hm;
  const int depth = (int)c->level_base.size() - 1;
  const u64 f0 = c->level_base[(size_t)depth - 1], f1 = c->level_base[(size_t)depth];
  const u64 F = f1 - f0;
  if (!F) {
    c->status = TLCG_DONE;
    return true;
  }
  const u64 d = distinct_of(c);
  const u64 worst = F * (u64)hm.max_new_per_state;
  const u64 est = next_level_estimate(c, F);
  if (!ensure_store(c, d + std::min(worst, std::max(est, (u64)1 << 20)))) return false;
  if ((c->opts.log2_fpset_slots <= 0 || c->opts.fpset_spill) && !ensure_fpset(c, d + est)) return false;
  if (!ensure_scratch(c, std::min(worst, dev_room(c, d)))) return false;
  for (;;) {
    if (!reset_ctr(c)) return false;
    HIPCHK_I(hipEventRecord(c->e0, c->stream));
    if (!launch_expand(c, f0, F, false)) return false;
    HIPCHK_I(hipEventRecord(c->e1, c->stream));
    if (c->opts.tlc_order) {
      // n_new is needed on the host to size the sort
      if (!read_ctr(c)) return false;
      if (!c->h_ctr->overflow && !tlc_order_level(c, c->h_ctr->n_new)) return false;
    }
    HIPCHK_I(hipEventRecord(c->e2, c->stream));
    if (!read_ctr(c)) return false;
    float ms_exp = 0, ms_all = 0;
    hipEventElapsedTime(&ms_exp, c->e0, c->e1);
    hipEventElapsedTime(&ms_all, c->e0, c->e2);
    c->expand_ms += ms_exp;
    c->kernel_ms += ms_all;
    const unsigned ovf = c->h_ctr->overflow;
    if (!ovf) break;
    if (ovf & OVF_WIDE_SPIN) {
      c->err = "internal: wide FPSet slot never published";
      return false;
    }
    // grow and redo the level from the committed levels
    ++c->levels_redone;
    if (ovf & OVF_STORE) {
      if (!ensure_store(c, d + std::max<u64>(c->h_ctr->n_new, 2 * dev_room(c, d)))) return false;
      if (!ensure_scratch(c, dev_room(c, d))) return false;
    }
    if (!regrow_fpset(c, ovf, d)) return false;
  }
  u64 n_new = c->h_ctr->n_new;
  if (c->opts.fpset_spill && (n_new = tier_filter_level(c, d, n_new)) == ~0ull) return false;
  c->gen_at.resize((size_t)depth - 1);
  c->gen_at.push_back(c->generated);
  c->generated += c->h_ctr->generated;
  if (c->outdeg_valid && !add_child_runs(c, d, n_new, F)) return false;
  if (n_new) c->level_base.push_back(d + n_new);
  const u64 uev = user_check_level(c, d, n_new, false);
  if (uev == ~0ull - 1) return false;
  const u64 ev = std::min<u64>(c->h_ctr->event, uev);
  if (ev != NO_EVENT) return resolve_event(c, ev, depth);
  if (!n_new) c->status = TLCG_DONE;
  return true;
}

}  // namespace

namespace tlcg {

void ctx_undo_expand(tlcg_ctx* c, tlcg_stats* st) {
  if (c->engine == TLCG_ENGINE_GLOBAL && !c->gen_at.empty() && c->pending == c->h_ctr->n_new) {
    c->generated = c->gen_at.back();
    c->gen_at.pop_back();
    c->pending = 0;
  }
  fill_stats(c, st);
}

// The counterexample of a multi-rank run (the parent references
// walked across the ranks' stores, host-mediated).  Collective: every rank of
// t calls it with the same `first` (the rank holding the first error,
// run_ranks); each hop's owner reads the state and its parent reference from
// its store and an all-reduce (sum; the other ranks add zeros) hands them to
// every rank.  A parent reference names its rank (bits 56..63), so the walk
// follows states absorbed from other ranks back to their discoverers.  On
// success every rank holds the trace (tlcg_trace_words); false only on a
// transport failure (a state the owner cannot read ends the walk: no trace).
bool trace_ranks(tlcg_ctx* c, Transport& t, int first, std::string* err) {
  const Layout& L = c->hm.L;
  const int me = t.rank(), w = c->words;
  const u64 ordmask = (1ull << L.ord_bits) - 1, refmask = (1ull << 56) - 1;
  // a trace the first rank already holds (the component tree's closed mode
  // replays the error's component, which lies on that rank): handed to all
  uint64_t held = me == first && c->xtrace_valid ? (uint64_t)c->xtrace_states.size() : 0;
  if (!t.allreduce(&held, 1, RED_SUM, err)) return false;
  if (held) {
    std::vector<uint64_t> buf((size_t)held * 3, 0);  // state words, action + 2
    if (me == first)
      for (size_t i = 0; i < (size_t)held; ++i) {
        split_words(c->xtrace_states[i], &buf[i * 3], 2);
        buf[i * 3 + 2] = (uint64_t)(c->xtrace_acts[i] + 2);
      }
    if (!t.allreduce(buf.data(), (int)buf.size(), RED_SUM, err)) return false;
    c->xtrace_states.assign((size_t)held, 0);
    c->xtrace_acts.assign((size_t)held, 0);
    for (size_t i = 0; i < (size_t)held; ++i) {
      c->xtrace_states[i] = join_words(&buf[i * 3], 2);
      c->xtrace_acts[i] = (int)buf[i * 3 + 2] - 2;
    }
    c->xtrace_valid = true;
    return true;
  }
  c->xtrace_valid = false;
  c->xtrace_states.clear();
  c->xtrace_acts.clear();
  // the event: level, status, action, its parent reference, the event state
  uint64_t ev[7] = {0, 0, 0, 0, 0, 0, 0};
  if (me == first) {
    u64 sw[2] = {0, 0};
    split_words(c->ev_state, sw, w);
    ev[0] = (u64)(c->ev_level + 1);
    ev[1] = (u64)c->status;
    ev[2] = (u64)(c->ev_action + 2);  // (TLCG_ACT_INIT = -1)
    ev[3] = c->ev_parent_gidx != NO_PARENT ? ((u64)c->opts.rank << 56) | (c->ev_parent_gidx << L.ord_bits)
                                           : c->ev_parent_ref;
    ev[4] = sw[0];
    ev[5] = sw[1];
    ev[6] = 1;
  }
  if (!t.allreduce(ev, 7, RED_SUM, err)) return false;
  if (ev[6] != 1 || ev[0] == 0) return true;  // (no event on `first`: no trace)
  u64 evw[2] = {ev[4], ev[5]};
  const u128 ev_state = join_words(evw, w);
  const int level = (int)ev[0] - 1, status = (int)ev[1], action = (int)ev[2] - 2;
  std::vector<u128> st;
  std::vector<int> act;
  if (level == 0) {
    st.push_back(ev_state);
    act.push_back(TLCG_ACT_INIT);
  } else {
    u64 ref = ev[3];
    for (int hop = 0;; ++hop) {
      if (ref == NO_PARENT || hop > (1 << 16)) return true;  // (a broken chain: no trace)
      const int owner = (int)(ref >> 56);
      const u64 g = (ref & refmask) >> L.ord_bits;
      uint64_t msg[4] = {0, 0, 0, 0};  // ok, parent reference, state words
      if (me == owner) {
        u128 s = 0;
        u64 p = 0;
        if (g < store_end(c) && state_at(c, g, &s, &p)) {
          u64 sw[2] = {0, 0};
          split_words(s, sw, w);
          msg[0] = 1;
          msg[1] = p;
          msg[2] = sw[0];
          msg[3] = sw[1];
        }
      }
      if (!t.allreduce(msg, 4, RED_SUM, err)) return false;
      if (msg[0] != 1) return true;
      u64 sw[2] = {msg[2], msg[3]};
      st.push_back(join_words(sw, w));
      if (msg[1] == NO_PARENT) {
        act.push_back(TLCG_ACT_INIT);
        break;
      }
      act.push_back(action_of_ordinal(L, (int)(msg[1] & ordmask)));
      ref = msg[1];
    }
    std::reverse(st.begin(), st.end());
    std::reverse(act.begin(), act.end());
    if (status == TLCG_VIOLATION || status == TLCG_INVARIANT_ERROR) {
      st.push_back(ev_state);
      act.push_back(action);
    }
  }
  c->xtrace_states = std::move(st);
  c->xtrace_acts = std::move(act);
  c->xtrace_valid = true;
  return true;
}

}  // namespace tlcg

extern "C" {

int tlcg_create(const tlcg_model* m, const tlcg_opts* o, tlcg_ctx** out) {
  if (!m || !out) return -1;
  *out = nullptr;
  tlcg_ctx* c = new tlcg_ctx();
  c->model = *m;
  if (o) c->opts = *o;
  else std::memset(&c->opts, 0, sizeof c->opts);
  if (c->opts.world <= 0) c->opts.world = 1;
  if (c->opts.world > 64 || c->opts.rank < 0 || c->opts.rank >= c->opts.world) {
    c->err = "rank/world out of range (world <= 64)";
    *out = c;
    return -2;
  }
  if (c->opts.tlc_order && c->opts.world != 1) {
    c->err = "TLC-order mode needs world == 1";
    *out = c;
    return -2;
  }
  if (!build_model(*m, &c->hm, &c->err)) {
    *out = c;
    return -3;
  }
  c->user_defs = m->user_defs ? m->user_defs : "";
  c->model.user_defs = m->user_defs ? c->user_defs.c_str() : nullptr;
  if (c->hm.user) c->user_src = user_device_source(*c->hm.user);
  c->words = state_words(c->hm.L);
  // partition key: `messages` alone when it is immutable (no Producer), so a
  // state's whole successor graph stays on its owner rank; else the state.
  const int part = c->opts.partition ? c->opts.partition : (c->hm.L.producer ? 2 : 1);
  c->owner_mask = part == 1 ? c->hm.L.msgs_mask : ~0ull;
  c->closed = c->opts.world == 1 || (part == 1 && !c->hm.L.producer);
  if (c->words == 2 && c->opts.world > 1 && (!c->closed || c->hm.L.msgs_mask_hi)) {
    c->err = "wide (> 63-bit) states are partitioned only by an immutable `messages` held in the low word "
             "(no Producer, partition 0/1)";
    *out = c;
    return -2;
  }
  if (c->opts.fpset_spill && c->words != 1) {
    c->err = "the host FPSet tier keeps <= 63-bit states";
    *out = c;
    return -2;
  }
  if (c->opts.engine == TLCG_ENGINE_TREE && !tree_applicable(c) && !tree_closed_applicable(c)) {
    c->err = "the component-tree engine needs a modelled Producer, one rank, <= 63-bit states, no TLC-order "
             "mode and no outdegree statistics";
    *out = c;
    return -2;
  }
  if (c->opts.engine == TLCG_ENGINE_COMPONENT && !component_applicable(c)) {
    c->err = "the component engine needs an immutable `messages` (no Producer), no TLC-order mode and a closed partition";
    *out = c;
    return -2;
  }
  *out = c;
  if (const char* v = getenv("TLCG_FAST_ITEMS")) c->fast_items = atoi(v);
  if (const char* v = getenv("TLCG_PROBE")) c->probe_mode = atoi(v);
  if (const char* v = getenv("TLCG_GRID")) c->grid_cap = (unsigned)atoi(v);
  if (c->fast_items != 0 && c->fast_items != 1 && c->fast_items != 2 && c->fast_items != 4) c->fast_items = 2;
  hipError_t e = hipSetDevice(c->opts.device);
  if (e != hipSuccess) {
    c->err = std::string("hipSetDevice: ") + hipGetErrorString(e);
    return -4;
  }
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreate(&c->e0) != hipSuccess || hipEventCreate(&c->e1) != hipSuccess ||
      hipEventCreate(&c->e2) != hipSuccess) {
    c->err = "stream/event creation failed";
    return -4;
  }
  if (hipMalloc((void**)&c->d_ctr, sizeof(LevelCtr)) != hipSuccess ||
      hipHostMalloc((void**)&c->h_ctr, sizeof(LevelCtr)) != hipSuccess ||
      hipMalloc((void**)&c->d_aux, sizeof(LevelCtr)) != hipSuccess ||
      hipHostMalloc((void**)&c->h_aux, sizeof(LevelCtr)) != hipSuccess) {
    c->err = "counter allocation failed";
    return -4;
  }
  if (c->hm.user && (hipMalloc((void**)&c->d_prog, sizeof(UserProg)) != hipSuccess ||
                     hipMemcpy(c->d_prog, c->hm.user.get(), sizeof(UserProg), hipMemcpyHostToDevice) != hipSuccess ||
                     hipMalloc((void**)&c->d_uev, sizeof(unsigned long long)) != hipSuccess)) {
    c->err = "user-invariant program upload failed";
    return -4;
  }
  if (c->opts.state_capacity && !ensure_store(c, c->opts.state_capacity)) return -5;
  if (c->opts.log2_fpset_slots > 0 && !rebuild_fpset(c, c->opts.log2_fpset_slots, 0)) return -5;
  return 0;
}

void tlcg_destroy(tlcg_ctx* c) {
  if (!c) return;
  const DeviceGuard dg(c);
  tlcg::comm_free(c->comm);
  c->comm = nullptr;
  if (c->stream) hipStreamSynchronize(c->stream);
  hipFree(c->d_slots);
  hipFree(c->d_dkey_slot);
  hipFree(c->d_states);
  hipFree(c->d_parents);
  free_tier(c);
  destroy_host_pool(c);
  hipFree(c->d_bloom);
  hipFree(c->d_q);
  hipFree(c->d_keep);
  hipFree(c->d_sel);
  hipFree(c->d_ftmp);
  hipFree(c->d_qn);
  hipFree(c->d_slot_new);
  hipFree(c->d_dk);
  hipFree(c->d_dk2);
  hipFree(c->d_st2);
  hipFree(c->d_sort_tmp);
  hipFree(c->d_outbox);
  hipFree(c->d_inbox);
  hipFree(c->d_ctr);
  hipFree(c->d_aux);
  hipFree(c->d_prog);
  hipFree(c->d_uev);
  tlcg_destroy(c->sub);
  c->sub = nullptr;
  jit_release(&c->jit);
  if (c->ujit_state == 1) jit_release_user_check(&c->ujit);
  hipFree(c->d_comp);
  hipFree(c->d_crec);
  hipFree(c->d_tree_dep);
  hipFree(c->d_tree_n);
  hipFree(c->d_tree_ctr);
  if (c->h_tree_ctr) hipHostFree(c->h_tree_ctr);
  hipFree(c->d_runs);
  hipFree(c->d_ovf[0]);
  hipFree(c->d_ovf[1]);
  if (c->h_comp) hipHostFree(c->h_comp);
  if (c->h_ctr) hipHostFree(c->h_ctr);
  if (c->h_aux) hipHostFree(c->h_aux);
  if (c->e0) hipEventDestroy(c->e0);
  if (c->e1) hipEventDestroy(c->e1);
  if (c->e2) hipEventDestroy(c->e2);
  if (c->stream) hipStreamDestroy(c->stream);
  delete c;
}

const char* tlcg_last_error(const tlcg_ctx* c) { return c ? c->err.c_str() : "null context"; }

void* tlcg_stream(tlcg_ctx* c) { return c ? (void*)c->stream : nullptr; }

int tlcg_init(tlcg_ctx* c, tlcg_stats* st) {
  const DeviceGuard dg(c);
  if (!c || !c->stream) return -1;
  free_tier(c);
  free_host_chunks(c);
  if (c->tlc_switched) {  // (the last run took TLC order for a tree error)
    c->opts.tlc_order = 0;
    c->tlc_switched = false;
  }
  c->tree_event = false;
  c->ev_comp = ~0ull;
  c->stop_cached = false;
  c->tree_codes = false;
  c->xtrace_valid = false;
  c->kernel_ms = c->expand_ms = 0;
  c->status = TLCG_RUNNING;
  c->ev_word = NO_EVENT;
  c->ev_level = -1;
  c->ev_parent_gidx = NO_PARENT;
  c->ev_action = -1;
  if ((c->opts.engine == TLCG_ENGINE_AUTO || c->opts.engine == TLCG_ENGINE_TREE) && tree_applicable(c)) {
    // the component-tree engine runs the whole BFS here; 0 = the global engine
    // takes the model (an error to report, a component past the capacity, memory)
    const int r = run_tree(c);
    if (r < 0) return -10;
    if (r == 1) {
      c->inited = true;
      fill_stats(c, st);
      return 0;
    }
    // an error to report, on one rank: the global engine runs in TLC order,
    // so its trace and TLC's stop statistics need no second run
    if (c->tree_event && c->opts.world == 1 && !c->opts.tlc_order) {
      c->opts.tlc_order = 1;
      c->tlc_switched = true;
    }
  }
  if (c->opts.engine != TLCG_ENGINE_GLOBAL && c->opts.engine != TLCG_ENGINE_TREE && component_applicable(c)) {
    // the component engine runs the whole BFS here; 0 = a component needs the global engine
    const int r = run_component(c);
    if (r < 0) return -10;
    if (r == 1) {
      c->inited = true;
      fill_stats(c, st);
      return 0;
    }
    if (c->opts.engine == TLCG_ENGINE_COMPONENT) {
      c->err = c->hm.user && !c->jit_used
                   ? "user invariants need the specialized kernels, which could not be built: " + c->jit_error
                   : "a component does not fit on chip (over 255 states or 48 levels); use the global engine";
      return -12;
    }
  }
  if ((c->opts.engine == TLCG_ENGINE_AUTO || c->opts.engine == TLCG_ENGINE_TREE) && tree_closed_applicable(c)) {
    // components too large for a lane: the component tree's closed mode
    const int r = run_tree(c);
    if (r < 0) return -10;
    if (r == 1) {
      c->inited = true;
      fill_stats(c, st);
      return 0;
    }
  }
  if (!run_init(c)) return -10;
  c->inited = true;
  fill_stats(c, st);
  return 0;
}

int tlcg_step_level(tlcg_ctx* c, tlcg_stats* st) {
  const DeviceGuard dg(c);
  if (!c || !c->inited) return -1;
  if (c->engine != TLCG_ENGINE_GLOBAL) {  // the on-chip engines finish the run in tlcg_init
    fill_stats(c, st);
    return 0;
  }
  if (!c->closed) {
    c->err = "successors can leave this rank: use tlcg_expand/outbox/inbox/absorb/end_level";
    return -2;
  }
  if (!step_level(c)) return -10;
  fill_stats(c, st);
  return 0;
}

int tlcg_run(tlcg_ctx* c, tlcg_stats* st) {
  int r = tlcg_init(c, st);
  if (r) return r;
  while (c->status == TLCG_RUNNING) {
    r = tlcg_step_level(c, st);
    if (r) return r;
  }
  fill_stats(c, st);
  return 0;
}

int tlcg_level_sizes(tlcg_ctx* c, uint64_t* out, int32_t cap, int32_t* n) {
  if (!c) return -1;
  if (c->engine != TLCG_ENGINE_GLOBAL) {
    const int depth = (int)c->comp_levels.size();
    for (int i = 0; i < depth && i < cap; ++i) out[i] = c->comp_levels[(size_t)i];
    if (n) *n = depth;
    return 0;
  }
  const int depth = c->level_base.empty() ? 0 : (int)c->level_base.size() - 1;
  for (int i = 0; i < depth && i < cap; ++i) out[i] = c->level_base[(size_t)i + 1] - c->level_base[(size_t)i];
  if (n) *n = depth;
  return 0;
}

int tlcg_state_at_words(tlcg_ctx* c, uint64_t gidx, uint64_t* state, uint64_t* parent_ref) {
  const DeviceGuard dg(c);
  if (!c || gidx >= store_end(c)) return -1;
  u128 s = 0;
  u64 p = 0;
  if (!state_at(c, gidx, &s, &p)) return -10;
  if (state) split_words(s, state, c->words);
  if (parent_ref) *parent_ref = p;
  return 0;
}

int tlcg_state_at(tlcg_ctx* c, uint64_t gidx, uint64_t* state, uint64_t* parent_ref) {
  if (c && c->words != 1) {
    c->err = "a wide (> 63-bit) state: use tlcg_state_at_words";
    return -2;
  }
  return tlcg_state_at_words(c, gidx, state, parent_ref);
}

int tlcg_copy_states_words(tlcg_ctx* c, uint64_t first, uint64_t n, uint64_t* out) {
  const DeviceGuard dg(c);
  if (!c || first + n > store_end(c)) return -1;
  const u64 w = c->words;
  if (c->engine == TLCG_ENGINE_COMPONENT) {  // record slots decoded here, word slots copied
    while (n) {
      u64 m = n;
      if (const tlcg_ctx::CompPass* ps = comp_code_pass(c, first)) {
        m = std::min<u64>(n, ps->store_base + component_store_slots(ps->n, ps->K) - first);
        std::vector<uint32_t> rec(m);
        if (hipMemcpy(rec.data(), c->d_crec + (first - ps->store_base), m * 4, hipMemcpyDeviceToHost) != hipSuccess) {
          c->err = "copy failed";
          return -10;
        }
        for (u64 i = 0; i < m; ++i) out[i] = comp_slot_decode(c, *ps, first + i, rec[i], nullptr);
      } else {
        for (const auto& ps : c->passes)  // up to the next record pass
          if (ps.codes && ps.store_base > first) m = std::min<u64>(m, ps.store_base - first);
        if (hipMemcpy(out, dev_state(c, first), m * 8 * w, hipMemcpyDeviceToHost) != hipSuccess) {
          c->err = "copy failed";
          return -10;
        }
      }
      out += m * w;
      first += m;
      n -= m;
    }
    return 0;
  }
  if (c->tree_codes) {  // component codes: decoded here
    std::vector<uint32_t> codes(n);
    if (n && hipMemcpy(codes.data(), reinterpret_cast<const uint32_t*>(c->d_states) + first, n * 4,
                       hipMemcpyDeviceToHost) != hipSuccess) {
      c->err = "copy failed";
      return -10;
    }
    for (u64 i = 0; i < n; ++i) split_words(tree_code_word(c, first + i, codes[i]), out + i * w, (int)w);
    return 0;
  }
  while (n && first < c->win) {  // spilled states
    const auto& h = chunk_of(c, first);
    const u64 m = std::min<u64>(n, h.g0 + h.n - first);
    std::memcpy(out, h.st + (first - h.g0) * w, m * 8 * w);
    out += m * w;
    first += m;
    n -= m;
  }
  if (n && hipMemcpy(out, dev_state(c, first), n * 8 * w, hipMemcpyDeviceToHost) != hipSuccess) {
    c->err = "copy failed";
    return -10;
  }
  return 0;
}

int tlcg_copy_states(tlcg_ctx* c, uint64_t first, uint64_t n, uint64_t* out) {
  if (c && c->words != 1) {
    c->err = "wide (> 63-bit) states: use tlcg_copy_states_words";
    return -2;
  }
  return tlcg_copy_states_words(c, first, n, out);
}

int tlcg_trace_words(tlcg_ctx* c, uint64_t* states, int32_t* actions, int32_t cap, int32_t* len) {
  const DeviceGuard dg(c);
  if (!c) return -1;
  if (c->xtrace_valid) {  // a multi-rank run's counterexample (trace_ranks)
    const int n = (int)c->xtrace_states.size();
    for (int i = 0; i < n && i < cap; ++i) {
      if (states) split_words(c->xtrace_states[(size_t)i], states + (size_t)i * c->words, c->words);
      if (actions) actions[i] = c->xtrace_acts[(size_t)i];
    }
    if (len) *len = n;
    return 0;
  }
  if (c->ev_word == NO_EVENT) {
    c->err = "no violation to trace";
    return -2;
  }
  const Layout& L = c->hm.L;
  const u64 ordmask = (1ull << L.ord_bits) - 1;
  std::vector<u128> st;
  std::vector<int> act;
  if (c->ev_level == 0) {
    st.push_back(c->ev_state);
    act.push_back(TLCG_ACT_INIT);
  } else {
    if (c->ev_parent_gidx == NO_PARENT) {
      c->err = "the trace crosses ranks: walk it with tlcg_state_at on each rank";
      return -3;
    }
    u64 g = c->ev_parent_gidx;
    for (;;) {
      u128 s;
      u64 p;
      if (!state_at(c, g, &s, &p)) return -10;
      st.push_back(s);
      if (p == NO_PARENT) {
        act.push_back(TLCG_ACT_INIT);
        break;
      }
      if ((p >> 56) != (u64)c->opts.rank) {
        c->err = "the trace crosses ranks";
        return -3;
      }
      act.push_back(action_of_ordinal(L, (int)(p & ordmask)));
      g = (p & ((1ull << 56) - 1)) >> L.ord_bits;
    }
    std::reverse(st.begin(), st.end());
    std::reverse(act.begin(), act.end());
    if (c->status == TLCG_VIOLATION || c->status == TLCG_INVARIANT_ERROR) {
      st.push_back(c->ev_state);
      act.push_back(c->ev_action);
    }
  }
  const int n = (int)st.size();
  for (int i = 0; i < n && i < cap; ++i) {
    if (states) split_words(st[(size_t)i], states + (size_t)i * c->words, c->words);
    if (actions) actions[i] = act[(size_t)i];
  }
  if (len) *len = n;
  return 0;
}

int tlcg_trace(tlcg_ctx* c, uint64_t* states, int32_t* actions, int32_t cap, int32_t* len) {
  if (c && c->words != 1) {
    c->err = "a wide (> 63-bit) state: use tlcg_trace_words";
    return -2;
  }
  return tlcg_trace_words(c, states, actions, cap, len);
}

}  // extern "C"

namespace {

// per-level sizes and generated counts of the on-chip engine's run over
// initial states [0, hi) alone, in a context of its own (this one's store,
// traces and counts stay as they are)
bool prefix_counts(tlcg_ctx* c, u64 hi, std::vector<u64>* pl, std::vector<u64>* pg) {
  tlcg_opts o = c->opts;
  o.world = 1;
  o.rank = 0;
  o.engine = c->engine;
  o.outdegree = 0;
  o.tlc_order = 0;
  o.state_capacity = 0;
  o.log2_fpset_slots = 0;
  tlcg_model m = c->model;
  tlcg_ctx* t = nullptr;
  if (tlcg_create(&m, &o, &t) != 0) {
    c->err = std::string("TLC stop statistics: ") + (t ? t->err : "tlcg_create failed");
    tlcg_destroy(t);
    return false;
  }
  t->range_hi = hi;
  t->comp_mult = c->comp_mult;  // (the tuned slot hashes: same code graph)
  t->tree_mult = c->tree_mult;
  t->tree_disp_mult = c->tree_disp_mult;
  std::copy(c->tree_disp, c->tree_disp + TREE_DISP, t->tree_disp);
  tlcg_stats st;
  const bool ok = tlcg_init(t, &st) == 0 && t->engine == c->engine;
  if (ok) {
    *pl = t->comp_levels;
    *pg = t->comp_level_gen;
  } else {
    c->err = "TLC stop statistics: the prefix run failed: " + t->err;
  }
  tlcg_destroy(t);
  return ok;
}

// TLC's stop statistics of an on-chip engine's error on a closed partition
// (replay_component): TLC's queue holds each level in component order, so
// at its stop TLC has generated and found everything of levels before the
// stopping state's, the components before the error's on the stopping
// level (a prefix run: initial states [0, comp)), and the error component's
// own share (its replay)
int onchip_stop_stats(tlcg_ctx* c, uint64_t* generated, uint64_t* distinct, uint64_t* left_on_queue) {
  const int E = c->ev_level;
  const u64 comp = c->ev_comp;
  if (E == 0) {  // an initial state: Init enumeration index comp, nothing dequeued yet
    *generated = *distinct = *left_on_queue = comp + 1;
    return 0;
  }
  CompReplay rp;
  if (!replay_component(c, comp, &rp) || rp.level != E) {
    c->err = "internal: the error's component replay disagrees with the engine";
    return -10;
  }
  std::vector<u64> pl, pg;
  if (comp > 0 && !prefix_counts(c, comp, &pl, &pg)) return -10;
  auto at = [](const std::vector<u64>& v, int i) -> u64 { return i >= 0 && (size_t)i < v.size() ? v[(size_t)i] : 0; };
  u64 gen = c->comp_init, dist = 0, before = 0;
  for (int l = 0; l < E - 1; ++l) {
    gen += at(c->comp_level_gen, l);
    before += at(c->comp_levels, l);
  }
  for (int l = 0; l <= E - 1; ++l) dist += at(c->comp_levels, l);
  gen += at(pg, E - 1) + rp.outdeg_before + rp.partial;
  dist += at(pl, E) + rp.found_next;
  const u64 pos = before + at(pl, E - 1) + rp.p_index;  // the stopping state's place in TLC's queue
  *generated = gen;
  *distinct = dist;
  *left_on_queue = dist - (pos + 1);
  return 0;
}

}  // namespace

// TLC's statistics at the moment a one-worker run stops on the error this
// context found (tlcgpu.h).  TLC's Worker dequeues states in FIFO order and,
// per state, runs the Next disjuncts in order: each action's successors are
// generated as one StateVec and counted (statesGenerated += its size) before
// any of them is put into the FPSet, enqueued and checked; the run stops at
// the first violating new state, at a failing action (before its successors
// are counted) or after all actions of a deadlocked state.  The global engine
// in TLC order stores states in exactly that FIFO order, a level sorted by
// first-discovery key (parent_gidx << ord_bits | ordinal), so:
//   generated = gen_at[d] + outdeg(level-d states before p) + p's successors
//               up to the stopping action;
//   distinct  = states of levels <= d + level-(d+1) states discovered before
//               the stop (a binary search over their parent references);
//   left on queue = distinct - (p + 1)  (p and everything before it dequeued).
int tlcg_tlc_stop_stats(tlcg_ctx* c, uint64_t* generated, uint64_t* distinct, uint64_t* left_on_queue) {
  const DeviceGuard dg(c);
  if (!c) return -1;
  if (c->stop_cached && c->status >= TLCG_VIOLATION) {  // (worked out with the run: producer_error)
    *generated = c->stop_g;
    *distinct = c->stop_d;
    *left_on_queue = c->stop_q;
    return 0;
  }
  if (c->status >= TLCG_VIOLATION && c->opts.world == 1 && c->engine != TLCG_ENGINE_GLOBAL && !c->hm.L.producer &&
      c->ev_comp != ~0ull)
    return onchip_stop_stats(c, generated, distinct, left_on_queue);
  if (c->status < TLCG_VIOLATION || !c->opts.tlc_order || c->opts.world != 1 || c->engine != TLCG_ENGINE_GLOBAL) {
    c->err = "TLC stop statistics need a global-engine run in TLC order, or an on-chip engine's run of a closed "
             "partition (world 1), that stopped on an error";
    return -2;
  }
  const Layout& L = c->hm.L;
  const u64 dkey = c->ev_word >> 6;
  const int kind = (int)((c->ev_word >> 4) & 3);
  if (c->ev_level == 0) {  // an initial state: Init enumeration index dkey, nothing dequeued yet
    *generated = *distinct = *left_on_queue = dkey + 1;
    return 0;
  }
  const size_t d = (size_t)c->ev_level - 1;  // level of the expanded state p
  if (c->gen_at.size() <= d || c->level_base.size() <= d + 1) {
    c->err = "TLC stop statistics are not available for a recovered run";
    return -2;
  }
  const u64 pg = c->ev_parent_gidx;
  const u64 f0 = c->level_base[d];
  // successors of p counted before the stop: ordinals [0, lim)
  const int a = c->ev_action;
  const int lim = kind == EVK_DEADLOCK ? L.nkv + N_ACTIONS - 1
                : kind == EVK_ACTION_ERROR ? ordinal_of(L, a, 0)
                : (a == ACT_PRODUCER ? L.nkv : ordinal_of(L, a, 0) + 1);
  u128 ps = 0;
  u64 pp = 0;
  if (!state_at(c, pg, &ps, &pp)) return -10;
  u64 partial = 0;
  for (int o = 0; o < lim; ++o) {
    u128 t = 0;
    partial += successor_at_any(c, ps, o, &t) == 1;
  }
  // out-degrees of the level-d states dequeued before p
  const u64 n = pg - f0, w = c->words;
  std::vector<u64> buf(std::max<u64>(n, 1) * w);
  if (n && tlcg_copy_states_words(c, f0, n, buf.data()) != 0) return -10;
  const int nt = (int)std::min<u64>(16, std::max<u64>(1, n / 65536));
  std::vector<u64> part((size_t)nt, 0);
  std::vector<std::thread> th;
  for (int t = 0; t < nt; ++t)
    th.emplace_back([&, t] {
      u64 acc = 0;
      for (u64 i = n * t / nt; i < n * (t + 1) / nt; ++i) {
        if (w == 1) {
          u64 out[80];
          acc += (u64)host_successors<u64>(L, buf[i], out, nullptr, 80);
        } else {
          u128 out[80];
          acc += (u64)host_successors<u128>(L, join_words(&buf[i * 2], 2), out, nullptr, 80);
        }
      }
      part[(size_t)t] = acc;
    });
  for (auto& x : th) x.join();
  u64 prefix = 0;
  for (u64 x : part) prefix += x;
  // level d + 1 (sorted by discovery key): states discovered before the stop
  const u64 n1 = c->level_base[d + 1];
  const u64 n2 = c->level_base.size() > d + 2 ? c->level_base[d + 2] : n1;
  const u64 key_mask = (1ull << 56) - 1;
  const u64 stop_key = kind == EVK_VIOLATION || kind == EVK_INV_ERROR ? dkey + 1 : (pg << L.ord_bits) | (u64)lim;
  u64 lo = n1, hi = n2;  // first index whose discovery key >= stop_key
  while (lo < hi) {
    const u64 mid = lo + (hi - lo) / 2;
    u128 s1 = 0;
    u64 p1 = 0;
    if (!state_at(c, mid, &s1, &p1)) return -10;
    if ((p1 & key_mask) < stop_key) lo = mid + 1;
    else hi = mid;
  }
  *generated = c->gen_at[d] + prefix + partial;
  *distinct = lo;
  *left_on_queue = lo - (pg + 1);
  return 0;
}

// States generated per level (tlcgpu.h): out[0] = initial states, out[k] =
// successors generated by expanding level k - 1.
int tlcg_level_generated(tlcg_ctx* c, uint64_t* out, int32_t cap, int32_t* n) {
  if (!c || !n) return -1;
  std::vector<u64> v;
  if (c->engine != TLCG_ENGINE_GLOBAL) {
    if (c->comp_levels.empty()) {
      *n = 0;
      return 0;
    }
    v.push_back(c->comp_init);
    // expanded levels: all of them on a complete run; 0..E-1 at an error in level E
    const size_t expanded = c->status == TLCG_DONE ? c->comp_levels.size() : c->comp_levels.size() - 1;
    for (size_t l = 0; l < expanded && l < c->comp_level_gen.size(); ++l) v.push_back(c->comp_level_gen[l]);
  } else {
    if (c->level_base.size() < 2) {
      *n = 0;
      return 0;
    }
    if (c->gen_at.size() + 2 < c->level_base.size()) {
      c->err = "per-level generated counts are not available for a recovered run";
      return -2;
    }
    if (c->gen_at.empty()) {
      v.push_back(c->generated);
    } else {
      v.push_back(c->gen_at[0]);
      for (size_t k = 1; k < c->gen_at.size(); ++k) v.push_back(c->gen_at[k] - c->gen_at[k - 1]);
      v.push_back(c->generated - c->gen_at.back());
    }
  }
  *n = (int32_t)v.size();
  for (size_t i = 0; i < v.size() && (int32_t)i < cap; ++i) out[i] = v[i];
  return 0;
}

// TLC's outdegree histogram of a completed check (tlcgpu.h)
int tlcg_outdegree(tlcg_ctx* c, uint64_t* hist, int32_t cap, int32_t* n) {
  if (!c || !n) return -1;
  if (c->status != TLCG_DONE || !c->outdeg_valid) {
    c->err = "the outdegree histogram needs tlcg_opts.outdegree and a completed check in TLC order or on the "
             "component engine";
    return -2;
  }
  size_t m = c->outdeg.size();
  while (m && c->outdeg[m - 1] == 0) --m;
  *n = (int32_t)m;
  for (size_t i = 0; i < m && (int32_t)i < cap; ++i) hist[i] = c->outdeg[i];
  return 0;
}

// ---- checkpoint / recover (TLC -checkpoint / -recover) ----
//
// File: CkptHeader, the tlcg_model, level_base[n_levels], then the committed
// states (d x words uint64) and the parent log (d uint64).  The FPSet is not
// saved: it is a function of the stored states and is rebuilt from them.
namespace {

struct CkptHeader {
  char magic[8];
  int32_t abi, words, rank, world, partition, tlc_order, status, pad;
  uint64_t n_levels, generated, levels_redone, distinct;
  double kernel_ms, expand_ms;
};
const char kCkptMagic[8] = {'T', 'L', 'C', 'G', 'C', 'K', 'P', '1'};
// the checkpoint's own format version (CkptHeader.abi), separate from the C
// ABI's: 2 = header, tlcg_model, levels, states, parents (rounds 1-2);
// 3 = the same with tlcg_model.user_defs as a length-prefixed text after the
// model (a C-ABI bump no longer orphans checkpoints)
constexpr int32_t kCkptFormat = 3;

bool same_constants(const tlcg_model& a, const tlcg_model& b) {
  if (std::string(a.user_defs ? a.user_defs : "") != std::string(b.user_defs ? b.user_defs : "")) return false;
  if (a.msg_sent_limit != b.msg_sent_limit || a.compaction_times_limit != b.compaction_times_limit ||
      a.consume_times_limit != b.consume_times_limit || a.max_crash_times != b.max_crash_times ||
      a.model_consumer != b.model_consumer || a.model_producer != b.model_producer ||
      a.retain_null_key != b.retain_null_key || a.check_deadlock != b.check_deadlock || a.n_keys != b.n_keys ||
      a.n_values != b.n_values || a.n_invariants != b.n_invariants)
    return false;
  for (int i = 0; i < a.n_keys; ++i)
    if (a.keys[i] != b.keys[i]) return false;
  for (int i = 0; i < a.n_values; ++i)
    if (a.values[i] != b.values[i]) return false;
  for (int i = 0; i < a.n_invariants; ++i)
    if (a.invariants[i] != b.invariants[i]) return false;
  return true;
}

// device <-> file through one pinned staging buffer
constexpr size_t kStage = 64u << 20;

bool dev_to_file(tlcg_ctx* c, FILE* f, const void* dev, size_t bytes, void* stage) {
  for (size_t off = 0; off < bytes; off += kStage) {
    const size_t n = std::min(kStage, bytes - off);
    HIPCHK(hipMemcpyAsync(stage, (const char*)dev + off, n, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    if (std::fwrite(stage, 1, n, f) != n) {
      c->err = "checkpoint write failed";
      return false;
    }
  }
  return true;
}

bool file_to_dev(tlcg_ctx* c, FILE* f, void* dev, size_t bytes, void* stage) {
  for (size_t off = 0; off < bytes; off += kStage) {
    const size_t n = std::min(kStage, bytes - off);
    if (std::fread(stage, 1, n, f) != n) {
      c->err = "checkpoint file is truncated";
      return false;
    }
    HIPCHK(hipMemcpyAsync((char*)dev + off, stage, n, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
  }
  return true;
}

}  // namespace

extern "C" {

int tlcg_checkpoint(tlcg_ctx* c, const char* path) {
  const DeviceGuard dg(c);
  if (!c || !path) return -1;
  if (!c->inited) {
    c->err = "nothing to checkpoint: call tlcg_init first";
    return -2;
  }
  if (c->engine != TLCG_ENGINE_GLOBAL) {
    c->err = "the on-chip engines (component engine, component tree) complete the whole check inside tlcg_init: "
             "nothing to checkpoint";
    return -2;
  }
  if (c->pending || (c->status != TLCG_RUNNING && c->status != TLCG_DONE)) {
    c->err = "a checkpoint is taken between levels of a run that has not stopped on an error";
    return -2;
  }
  const u64 d = distinct_of(c);
  CkptHeader h;
  std::memset(&h, 0, sizeof h);
  std::memcpy(h.magic, kCkptMagic, 8);
  h.abi = kCkptFormat;
  h.words = c->words;
  h.rank = c->opts.rank;
  h.world = c->opts.world;
  h.partition = c->opts.partition;
  h.tlc_order = c->opts.tlc_order;
  h.status = c->status;
  h.n_levels = c->level_base.size();
  h.generated = c->generated;
  h.levels_redone = c->levels_redone;
  h.distinct = d;
  h.kernel_ms = c->kernel_ms;
  h.expand_ms = c->expand_ms;
  const std::string tmp = std::string(path) + ".tmp";
  FILE* f = std::fopen(tmp.c_str(), "wb");
  if (!f) {
    c->err = std::string("cannot write ") + tmp;
    return -3;
  }
  c->err.clear();
  void* stage = nullptr;
  bool ok = hipHostMalloc(&stage, kStage) == hipSuccess;
  tlcg_model mw = c->model;
  mw.user_defs = nullptr;  // (the text follows the model)
  const uint64_t ulen = c->user_defs.size();
  ok = ok && std::fwrite(&h, sizeof h, 1, f) == 1 && std::fwrite(&mw, sizeof mw, 1, f) == 1 &&
       std::fwrite(&ulen, 8, 1, f) == 1 && std::fwrite(c->user_defs.data(), 1, ulen, f) == ulen &&
       std::fwrite(c->level_base.data(), 8, c->level_base.size(), f) == c->level_base.size();
  // spilled levels from their host chunks, the rest from the device
  for (const auto& hc : c->hchunks) ok = ok && std::fwrite(hc.st, 8 * c->words, hc.n, f) == hc.n;
  ok = ok && dev_to_file(c, f, c->d_states, (d - c->win) * 8 * c->words, stage);
  for (const auto& hc : c->hchunks) ok = ok && std::fwrite(hc.par, 8, hc.n, f) == hc.n;
  ok = ok && dev_to_file(c, f, c->d_parents, (d - c->win) * 8, stage);
  if (stage) hipHostFree(stage);
  ok = (std::fclose(f) == 0) && ok;
  if (!ok || std::rename(tmp.c_str(), path) != 0) {
    if (c->err.empty()) c->err = std::string("checkpoint to ") + path + " failed";
    std::remove(tmp.c_str());
    return -3;
  }
  return 0;
}

int tlcg_recover(tlcg_ctx* c, const char* path, tlcg_stats* st) {
  const DeviceGuard dg(c);
  if (!c || !path) return -1;
  FILE* f = std::fopen(path, "rb");
  if (!f) {
    c->err = std::string("cannot read checkpoint ") + path;
    return -3;
  }
  CkptHeader h;
  tlcg_model m;
  if (std::fread(&h, sizeof h, 1, f) != 1 || std::memcmp(h.magic, kCkptMagic, 8) != 0 ||
      std::fread(&m, sizeof m, 1, f) != 1) {
    std::fclose(f);
    c->err = std::string(path) + " is not a tlcgpu checkpoint";
    return -3;
  }
  if (h.abi != kCkptFormat) {
    std::fclose(f);
    c->err = "the checkpoint is in format " + std::to_string(h.abi) + "; this build reads format " +
             std::to_string(kCkptFormat);
    return -4;
  }
  uint64_t ulen = 0;
  std::string udefs;
  if (std::fread(&ulen, 8, 1, f) != 1 || ulen > (64u << 20)) {
    std::fclose(f);
    c->err = "checkpoint file is truncated or corrupt";
    return -3;
  }
  udefs.resize(ulen);
  if (ulen && std::fread(&udefs[0], 1, ulen, f) != ulen) {
    std::fclose(f);
    c->err = "checkpoint file is truncated or corrupt";
    return -3;
  }
  m.user_defs = ulen ? udefs.c_str() : nullptr;
  if (!same_constants(m, c->model) || h.words != c->words || h.rank != c->opts.rank ||
      h.world != c->opts.world || h.tlc_order != c->opts.tlc_order ||
      (h.world > 1 && h.partition != c->opts.partition) || h.n_levels < 1) {
    std::fclose(f);
    c->err = "the checkpoint was taken for other constants or options";
    return -4;
  }
  // the header's sizes must match the file before anything is sized from
  // them: level bases (8 B each), then states (8 B x words) and parent refs
  // (8 B) of every distinct state
  const long body = std::ftell(f);
  std::fseek(f, 0, SEEK_END);
  const long fsize = std::ftell(f);
  std::fseek(f, body, SEEK_SET);
  const u64 avail = body >= 0 && fsize > body ? (u64)(fsize - body) : 0;
  const u64 per_state = 8 * (u64)c->words + 8;
  if (h.n_levels > avail / 8 || h.distinct > avail / per_state || h.n_levels * 8 + h.distinct * per_state != avail) {
    std::fclose(f);
    c->err = "checkpoint file is truncated or corrupt (its sizes do not match the file)";
    return -3;
  }
  std::vector<u64> lb(h.n_levels);
  bool lb_ok = std::fread(lb.data(), 8, lb.size(), f) == lb.size() && lb[0] == 0 && lb.back() == h.distinct;
  for (size_t i = 1; lb_ok && i < lb.size(); ++i) lb_ok = lb[i] >= lb[i - 1];
  if (!lb_ok) {
    std::fclose(f);
    c->err = "checkpoint file is truncated or corrupt (level bases)";
    return -3;
  }
  // the run restarts on the global engine with exactly the committed levels
  c->engine = TLCG_ENGINE_GLOBAL;
  c->passes.clear();
  c->level_base.clear();
  c->pending = 0;
  c->err.clear();
  free_host_chunks(c);
  const u64 d = h.distinct, w = c->words;
  // with opts.spill the levels below the frontier go straight to host memory
  const u64 f0 = c->opts.spill && lb.size() >= 2 ? lb[lb.size() - 2] : 0;
  tlcg_ctx::HostChunk hc{0, f0, nullptr, nullptr};
  void* stage = nullptr;
  bool ok = hipHostMalloc(&stage, kStage) == hipSuccess;
  if (ok && f0) {
    hc.st = (u64*)host_block(c, f0 * 8 * w);
    hc.par = hc.st ? (u64*)host_block(c, f0 * 8) : nullptr;
    ok = hc.par != nullptr;
    if (!ok) {
      host_release(c, hc.st);
      c->err = "out of pinned host memory for the spilled levels";
    } else {
      c->hchunks.push_back(hc);
      c->win = f0;
    }
  }
  const u64 dn = d - f0;
  ok = ok && ensure_store(c, d + (dn >> 3) + (1u << 16));
  ok = ok && (!f0 || std::fread(hc.st, 8 * w, f0, f) == f0) && file_to_dev(c, f, c->d_states, dn * 8 * w, stage) &&
       (!f0 || std::fread(hc.par, 8, f0, f) == f0) && file_to_dev(c, f, c->d_parents, dn * 8, stage);
  if (stage) hipHostFree(stage);
  std::fclose(f);
  if (!ok) {
    if (c->err.empty()) c->err = "checkpoint file is truncated";
    return -10;
  }
  c->level_base = lb;
  c->gen_at.clear();  // (not in the checkpoint: tlcg_tlc_stop_stats refuses after a recover)
  c->outdeg_valid = false;  // (nor the outdegree histogram of the levels before it)
  c->generated = h.generated;
  c->levels_redone = h.levels_redone;
  c->kernel_ms = h.kernel_ms;
  c->expand_ms = h.expand_ms;
  c->status = h.status == TLCG_DONE ? TLCG_DONE : TLCG_RUNNING;
  c->ev_word = NO_EVENT;
  c->ev_level = -1;
  c->ev_parent_gidx = NO_PARENT;
  c->ev_parent_ref = NO_PARENT;
  c->ev_action = -1;
  // the FPSet is a function of the stored states: rebuild it from them
  free_tier(c);
  int l = c->opts.log2_fpset_slots > 0 ? c->opts.log2_fpset_slots : std::max(c->log2, 16);
  while (c->opts.log2_fpset_slots <= 0 && (1ull << l) < 2 * d && l < 40) ++l;
  if (c->opts.fpset_spill && l > fpset_max_log2(c)) {
    // the host tier takes the committed states, half a table at a time
    if (!rebuild_fpset(c, fpset_max_log2(c), 0)) return -10;
    while (c->t0_base < d)
      if (!flush_tier(c, std::min<u64>(d, c->t0_base + (1ull << c->log2) / 2))) return -10;
    l = c->log2;
  }
  if (!rebuild_fpset(c, l, d)) return -10;
  c->inited = true;
  fill_stats(c, st);
  return 0;
}

int tlcg_jit_selftest(const tlcg_model* m, const char* arch, char* err, int32_t cap) {
  HostModel hm;
  std::string e;
  if (!m || !build_model(*m, &hm, &e)) return -1;
  std::vector<char> code;
  if (!jit_compile(hm.L, arch ? arch : "gfx950", &code, &e, hm.user ? user_device_source(*hm.user) : "")) {
    if (err && cap > 0) std::snprintf(err, (size_t)cap, "%s", e.c_str());
    return -2;
  }
  // (user invariants: the global engine's check module too)
  std::vector<char> check;
  if (hm.user && !jit_compile(hm.L, arch ? arch : "gfx950", &check, &e, user_device_source(*hm.user), true)) {
    if (err && cap > 0) std::snprintf(err, (size_t)cap, "user-check module: %s", e.c_str());
    return -2;
  }
  if (err && cap > 0) err[0] = 0;
  return (int)(code.size() + check.size());
}

// Let devices 0..n-1 read and write each other's memory (xGMI peer access),
// for contexts of one process on several devices that exchange records by
// device-to-device copies.  Returns the number of pairs enabled.
int tlcg_peer_access(int32_t n) {
  int cur = 0, count = 0, pairs = 0;
  if (hipGetDevice(&cur) != hipSuccess || hipGetDeviceCount(&count) != hipSuccess) return -1;
  n = std::min(n, count);
  for (int a = 0; a < n; ++a) {
    if (hipSetDevice(a) != hipSuccess) continue;
    for (int b = 0; b < n; ++b) {
      int can = 0;
      if (a == b || hipDeviceCanAccessPeer(&can, a, b) != hipSuccess || !can) continue;
      const hipError_t e = hipDeviceEnablePeerAccess(b, 0);
      if (e == hipSuccess || e == hipErrorPeerAccessAlreadyEnabled) ++pairs;
      (void)hipGetLastError();
    }
  }
  (void)hipSetDevice(cur);
  return pairs;
}

int tlcg_device_count(void) {
  int n = 0;
  return hipGetDeviceCount(&n) == hipSuccess ? n : 0;
}

int tlcg_owner(tlcg_ctx* c, uint64_t state) {
  if (!c) return -1;  // wide states: pass the low word (the partition key lies there)
  return owner_hash(state & c->owner_mask, c->opts.world);
}

// ---- partitioned levels (world > 1) ----

int tlcg_expand(tlcg_ctx* c, tlcg_stats* st) {
  const DeviceGuard dg(c);
  if (!c || !c->inited) return -1;
  // a finished rank returns its stats, whichever engine finished it (an
  // on-chip engine completes this rank's share inside tlcg_init: ADVICE r3)
  if (c->status != TLCG_RUNNING) {
    fill_stats(c, st);
    return 0;
  }
  if (c->engine != TLCG_ENGINE_GLOBAL) {
    c->err = "the on-chip engine completed this rank's share in tlcg_init: there is no level to expand "
             "(tlcg_opts.engine = TLCG_ENGINE_GLOBAL for the exchange)";
    return -2;
  }
  const HostModel& hm = c->hm;
  const int depth = (int)c->level_base.size() - 1;
  const u64 f0 = depth ? c->level_base[(size_t)depth - 1] : 0;
  const u64 F = depth ? c->level_base[(size_t)depth] - f0 : 0;
  const u64 d = distinct_of(c);
  const u64 est = next_level_estimate(c, F);
  const u64 worst = F * (u64)hm.max_new_per_state;
  c->pending = 0;
  if (!ensure_store(c, d + std::min(worst, std::max(est, (u64)1 << 20)))) return -10;
  if ((c->opts.log2_fpset_slots <= 0 || c->opts.fpset_spill) && !ensure_fpset(c, d + est)) return -10;
  // outbox: an even split of the expected successors, with slack, at least a
  // share of the planned store (opts.state_capacity); it only grows, doubling
  // (a hipFree / hipMalloc between levels stalls every queue of the device,
  // the other ranks' kernels included)
  u64 per_dst = F ? 2 * est / (u64)c->opts.world + 1024 : 1024;
  per_dst = std::max<u64>(per_dst, c->opts.state_capacity / (2 * (u64)c->opts.world));
  if (per_dst > c->outbox_cap) per_dst = std::max<u64>(per_dst, 2 * c->outbox_cap);
  for (;;) {
    if (per_dst > c->outbox_cap) {
      hipFree(c->d_outbox);
      c->d_outbox = nullptr;
      c->outbox_cap = 0;
      if (!alloc_bytes(c, (void**)&c->d_outbox, per_dst * 16 * (u64)c->opts.world, "outbox")) return -10;
      c->outbox_cap = per_dst;
    }
    if (!reset_ctr(c)) return -10;
    if (F) {
      if (hipEventRecord(c->e0, c->stream) != hipSuccess) return -10;
      if (!launch_expand(c, f0, F, true)) return -10;
      if (hipEventRecord(c->e1, c->stream) != hipSuccess) return -10;
    }
    if (!read_ctr(c)) return -10;
    if (F) {
      float ms = 0;
      hipEventElapsedTime(&ms, c->e0, c->e1);
      c->expand_ms += ms;
      c->kernel_ms += ms;
    }
    const unsigned ovf = c->h_ctr->overflow;
    if (!ovf) break;
    if (std::getenv("TLCG_RANK_TRACE"))
      std::fprintf(stderr, "rank %d level %d: expand overflow %u (outbox cap %llu, store room %llu, log2 %d)\n",
                   c->opts.rank, depth, ovf, (unsigned long long)c->outbox_cap, (unsigned long long)dev_room(c, d),
                   c->log2);
    // grow what overflowed and redo the expansion from the committed levels
    ++c->levels_redone;
    if (ovf & OVF_OUTBOX) {
      u64 mx = 0;
      for (int r = 0; r < c->opts.world; ++r) mx = std::max<u64>(mx, c->h_ctr->n_out[r]);
      per_dst = std::max<u64>(2 * per_dst, mx + mx / 4);
    }
    if ((ovf & OVF_STORE) && !ensure_store(c, d + std::max<u64>(c->h_ctr->n_new, 2 * dev_room(c, d)))) return -10;
    if (!regrow_fpset(c, ovf, d)) return -10;
  }
  c->gen_at.resize((size_t)depth - 1);
  c->gen_at.push_back(c->generated);
  c->generated += c->h_ctr->generated;
  c->pending = c->h_ctr->n_new;
  fill_stats(c, st);
  return 0;
}

int tlcg_outbox(tlcg_ctx* c, int32_t dst, void** dev_records, uint64_t* n_records) {
  if (!c || dst < 0 || dst >= c->opts.world) return -1;
  if (dev_records) *dev_records = c->d_outbox ? (void*)(c->d_outbox + 2 * (u64)dst * c->outbox_cap) : nullptr;
  if (n_records) *n_records = dst == c->opts.rank ? 0 : c->h_ctr->n_out[dst];
  return 0;
}

int tlcg_inbox(tlcg_ctx* c, uint64_t n_records, void** dev_records) {
  const DeviceGuard dg(c);
  if (!c) return -1;
  if (n_records > c->inbox_cap) {
    hipFree(c->d_inbox);
    c->d_inbox = nullptr;
    // doubling, from a share of the planned store (see the outbox in tlcg_expand)
    u64 ncap = std::max<u64>({n_records + n_records / 4, 4096, 2 * c->inbox_cap, c->opts.state_capacity / 8});
    c->inbox_cap = 0;
    if (!alloc_bytes(c, (void**)&c->d_inbox, ncap * 16, "inbox")) return -10;
    c->inbox_cap = ncap;
  }
  if (dev_records) *dev_records = c->d_inbox;
  return 0;
}

int tlcg_absorb(tlcg_ctx* c, uint64_t n_records, tlcg_stats* st) {
  const DeviceGuard dg(c);
  if (!c || n_records > c->inbox_cap) return -1;
  if (c->status != TLCG_RUNNING || !n_records) {
    fill_stats(c, st);
    return 0;
  }
  const u64 d = distinct_of(c);
  const u64 local_new = c->h_ctr->n_new;  // appended by the expand (ctr not reset)
  const LevelCtr before = *c->h_ctr;      // the level's counters after the expand
  c->pending = local_new;
  if (!ensure_store(c, d + local_new + n_records)) return -10;
  if ((c->opts.log2_fpset_slots <= 0 || c->opts.fpset_spill) && !ensure_fpset(c, d + local_new + n_records))
    return -10;
  for (;;) {
    if (hipEventRecord(c->e0, c->stream) != hipSuccess) return -10;
    k_absorb<<<grid_for(n_records, (u64)BLOCK * ABSORB_IT, 0x7fffffffu), BLOCK, 0, c->stream>>>(
        c->hm.L, c->d_inbox, n_records, c->d_slots, c->log2, dev_state(c, d), dev_parent(c, d), dev_room(c, d),
        c->d_ctr);
    if (hipGetLastError() != hipSuccess) return -10;
    if (hipEventRecord(c->e1, c->stream) != hipSuccess) return -10;
    if (!read_ctr(c)) return -10;
    float ms = 0;
    hipEventElapsedTime(&ms, c->e0, c->e1);
    c->kernel_ms += ms;
    const unsigned ovf = c->h_ctr->overflow;
    if (!ovf) break;
    if (std::getenv("TLCG_RANK_TRACE"))
      std::fprintf(stderr, "rank %d: absorb overflow %u (records %llu, store room %llu, log2 %d)\n", c->opts.rank,
                   ovf, (unsigned long long)n_records, (unsigned long long)dev_room(c, d), c->log2);
    // grow and redo: forget this absorb's appends and inserts
    ++c->levels_redone;
    if ((ovf & OVF_STORE) && !ensure_store(c, d + local_new + n_records)) return -10;
    if (!regrow_fpset(c, ovf, d + local_new)) return -10;
    *c->h_ctr = before;
    if (hipMemcpyAsync(c->d_ctr, c->h_ctr, sizeof(LevelCtr), hipMemcpyHostToDevice, c->stream) != hipSuccess)
      return -10;
  }
  c->pending = c->h_ctr->n_new;
  fill_stats(c, st);
  return 0;
}

// Copy the first n records for `dst` to caller memory (host or device; the
// runtime infers which), ordered after the expand on the context's stream.
int tlcg_outbox_read(tlcg_ctx* c, int32_t dst, void* out, uint64_t n) {
  const DeviceGuard dg(c);
  if (!c || dst < 0 || dst >= c->opts.world || dst == c->opts.rank) return -1;
  if (!n) return 0;
  if (!c->d_outbox || n > c->h_ctr->n_out[dst] || n > c->outbox_cap) return -1;
  HIPCHK_I(hipMemcpyAsync(out, c->d_outbox + 2 * (u64)dst * c->outbox_cap, n * 16, hipMemcpyDefault, c->stream));
  HIPCHK_I(hipStreamSynchronize(c->stream));
  return 0;
}

// Every destination's records, destination-major in rank order (this rank's
// own, always empty, skipped), copied to one caller buffer with one stream
// synchronization: the send buffer of an all-to-all.
int tlcg_outbox_gather(tlcg_ctx* c, void* out) {
  const DeviceGuard dg(c);
  if (!c) return -1;
  u64 off = 0;
  for (int dst = 0; dst < c->opts.world; ++dst) {
    if (dst == c->opts.rank) continue;
    const u64 n = c->h_ctr->n_out[dst];
    if (!n) continue;
    if (!c->d_outbox || n > c->outbox_cap) return -1;
    HIPCHK_I(hipMemcpyAsync((char*)out + off * 16, c->d_outbox + 2 * (u64)dst * c->outbox_cap, n * 16,
                            hipMemcpyDefault, c->stream));
    off += n;
  }
  HIPCHK_I(hipStreamSynchronize(c->stream));
  return 0;
}

// tlcg_inbox + copy + tlcg_absorb in one call: the copy of the caller's
// records (host or device) and the insert run in order on the context's stream.
int tlcg_absorb_records(tlcg_ctx* c, const void* records, uint64_t n, tlcg_stats* st) {
  const DeviceGuard dg(c);
  if (!c) return -1;
  if (n) {
    const int r = tlcg_inbox(c, n, nullptr);
    if (r) return r;
    HIPCHK_I(hipMemcpyAsync(c->d_inbox, records, n * 16, hipMemcpyDefault, c->stream));
  }
  return tlcg_absorb(c, n, st);
}

// The exchange of one process driving every rank (contexts on devices of one
// node, peer access enabled): each destination's inbox receives the records
// of every source, source-rank-major (the order an all-to-all delivers), by
// device-to-device copies over xGMI on the source streams.  Returns with all
// copies landed; n_in[d] = records now in ctxs[d]'s inbox, for tlcg_absorb.
int tlcg_exchange_local(tlcg_ctx* const* ctxs, int32_t n, uint64_t* n_in) {
  if (!ctxs || n < 1 || !n_in) return -1;
  for (int r = 0; r < n; ++r)
    if (!ctxs[r] || ctxs[r]->opts.world != n || ctxs[r]->opts.rank != r) return -1;
  for (int dst = 0; dst < n; ++dst) {
    tlcg_ctx* c = ctxs[dst];
    u64 total = 0;
    for (int src = 0; src < n; ++src)
      if (src != dst) total += ctxs[src]->h_ctr->n_out[dst];
    n_in[dst] = total;
    if (!total) continue;
    const int r = tlcg_inbox(c, total, nullptr);  // sized before any copy lands in it
    if (r) return r;
  }
  for (int src = 0; src < n; ++src) {
    tlcg_ctx* c = ctxs[src];
    const DeviceGuard dg(c);
    for (int dst = 0; dst < n; ++dst) {
      if (dst == src) continue;
      u64 at = 0;
      for (int s = 0; s < src; ++s)
        if (s != dst) at += ctxs[s]->h_ctr->n_out[dst];
      const u64 k = c->h_ctr->n_out[dst];
      if (!k) continue;
      if (!c->d_outbox || k > c->outbox_cap) return -1;
      HIPCHK_I(hipMemcpyPeerAsync(ctxs[dst]->d_inbox + 2 * at, ctxs[dst]->opts.device,
                                  c->d_outbox + 2 * (u64)dst * c->outbox_cap, c->opts.device, k * 16, c->stream));
    }
  }
  for (int src = 0; src < n; ++src) {
    tlcg_ctx* c = ctxs[src];
    const DeviceGuard dg(c);
    HIPCHK_I(hipStreamSynchronize(c->stream));
  }
  return 0;
}

int tlcg_partition_closed(const tlcg_ctx* c) { return c ? (int)c->closed : -1; }

int tlcg_end_level(tlcg_ctx* c, tlcg_stats* st) {
  const DeviceGuard dg(c);
  if (!c) return -1;
  if (c->status == TLCG_RUNNING) {
    const int depth = (int)c->level_base.size() - 1;
    const u64 d = distinct_of(c);
    u64 n_new = c->h_ctr->n_new;
    if (c->opts.fpset_spill && (n_new = tier_filter_level(c, d, n_new)) == ~0ull) return -10;
    c->level_base.push_back(d + n_new);  // empty levels kept (see run_init)
    c->pending = 0;
    // the user invariants on the level's new states, the absorbed ones included
    const u64 uev = user_check_level(c, d, n_new, false);
    if (uev == ~0ull - 1) return -10;
    const u64 ev = std::min<u64>(c->h_ctr->event, uev);
    if (ev != NO_EVENT) {
      if (!resolve_event(c, ev, depth)) return -10;
    }
  }
  fill_stats(c, st);
  return 0;
}

}  // extern "C"
