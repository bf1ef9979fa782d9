// pulsar-tlaplus_amd/csrc/kernels.h -- device-side building blocks of the
// BFS level: FPSet insert, LDS staging, the per-level counter block.
#pragma once
#if !defined(__HIPCC_RTC__)
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "model.h"
#endif

namespace tlcg {

constexpr int BLOCK = 256;        // 4 waves of 64
constexpr int ITEMS = 4;          // parents per thread per chunk (no Producer)
constexpr int STAGE_CAP = 2048;   // LDS staging entries per block (>= BLOCK * ITEMS * 2)
constexpr int MAX_PROBE = 4096;   // FPSet linear-probe limit before "grow and redo"
constexpr u64 SLOT_TAG = 1ull << 63;  // occupied-slot tag: slot = state | SLOT_TAG
constexpr u64 NO_EVENT = ~0ull;
constexpr u64 NO_PARENT = ~0ull;

// event kinds (an event stops the run, like TLC's first error)
enum EventKind { EVK_VIOLATION = 0, EVK_INV_ERROR = 1, EVK_DEADLOCK = 2, EVK_ACTION_ERROR = 3 };
// overflow flags
enum Overflow { OVF_FPSET = 1, OVF_STORE = 2, OVF_OUTBOX = 4, OVF_DUP_INIT = 8, OVF_WIDE_SPIN = 16 };

// per-level counter block, zeroed (event = ~0) before every level
struct LevelCtr {
  unsigned long long n_new;
  unsigned long long generated;
  unsigned long long event;       // min over (dkey << 6 | kind << 4 | index)
  unsigned int overflow;
  unsigned int pad;
  unsigned long long n_out[64];   // outbox records per destination rank
};

// event word: dkey = parent_gidx << ord_bits | ordinal (< 2^58), or the
// initial-state index for level 0.
TLCG_HD u64 make_event(u64 dkey, int kind, int index) {
  return (dkey << 6) | ((u64)kind << 4) | (u64)(index & 15);
}

// FPSet.put over an open-addressing table of 2^log2 8-byte slots.  A slot
// holds 0 (empty) or state|SLOT_TAG.  Slots only ever go 0 -> key, so a plain
// (possibly stale) load that sees a key is exact, and a stale 0 is resolved by
// the device-scope CAS.  Returns 1 inserted, 0 present, -1 probe limit.
//
// Wide states (u128, <= 126 bits): 16-byte slots {hi, lo}.  hi carries the
// state's bits 64..125 | SLOT_TAG, and WIDE_READY once lo is published.  An
// insert claims hi with a 64-bit CAS (0 -> hi), publishes lo with an atomic
// exchange, waits for it, then sets WIDE_READY; a prober whose hi matches waits
// for WIDE_READY and compares lo.  Every access after the claim is a
// device-scope atomic, performed at the memory side, so no XCD's L2 can serve a
// stale half.  Slots only go 0 -> hi -> hi|READY, so a stale plain first load
// is harmless (0 -> the CAS decides; hi without READY -> the wait re-reads).
constexpr u64 WIDE_READY = 1ull << 62;
constexpr int WIDE_SPIN = 1 << 22;  // bound on the wait for a publisher (then OVF_WIDE_SPIN)

template <typename W>
__device__ __forceinline__ int fpset_put(u64* __restrict__ slots, int log2, W state, u64 fp, u64* slot_out) {
  const u64 mask = (1ull << log2) - 1;
  u64 i = fp >> (64 - log2);
  if constexpr (sizeof(W) == 8) {
    const u64 key = state | SLOT_TAG;
#pragma unroll 1
    for (int p = 0; p < MAX_PROBE; ++p) {
      u64 v = __builtin_nontemporal_load(&slots[i]);
      if (v == key) { *slot_out = i; return 0; }
      if (v == 0) {
        u64 old = atomicCAS((unsigned long long*)&slots[i], 0ull, (unsigned long long)key);
        if (old == 0) { *slot_out = i; return 1; }
        if (old == key) { *slot_out = i; return 0; }
      }
      i = (i + 1) & mask;
    }
    return -1;
  } else {
    // The probe is a wave-uniform loop (it runs while ANY lane is unsettled)
    // so that a lane waiting on a slot that another lane of its own wave has
    // just claimed cannot spin ahead of that lane's publish: both happen in
    // the same trip.
    const u64 hi = (u64)(state >> 64) | SLOT_TAG, lo = (u64)state;
    enum { PROBING, CLAIMED, WAITING, SETTLED };
    int st = PROBING, res = -1, probes = 0, spins = 0;
    while (__any(st != SETTLED)) {
      unsigned long long* sl = (unsigned long long*)&slots[2 * i];
      if (st == PROBING) {
        u64 v = __builtin_nontemporal_load(&slots[2 * i]);
        if (v == 0) {
          v = atomicCAS(&sl[0], 0ull, (unsigned long long)hi);
          if (v == 0) st = CLAIMED;
        }
        if (st == PROBING) {
          if ((v & ~WIDE_READY) == hi) {
            st = WAITING;  // the same high half: compare the low half once published
          } else if (++probes >= MAX_PROBE) {
            st = SETTLED;
          } else {
            i = (i + 1) & mask;
          }
        }
      }
      if (st == CLAIMED) {  // publish lo, wait for it, then mark the slot ready
        atomicExch(&sl[1], (unsigned long long)lo);
        __builtin_amdgcn_s_waitcnt(0);
        atomicOr(&sl[0], (unsigned long long)WIDE_READY);
        st = SETTLED;
        res = 1;
      } else if (st == WAITING) {
        if (atomicOr(&sl[0], 0ull) & WIDE_READY) {
          if (atomicOr(&sl[1], 0ull) == lo) {
            st = SETTLED;
            res = 0;
          } else if (++probes >= MAX_PROBE) {
            st = SETTLED;
          } else {
            st = PROBING;
            i = (i + 1) & mask;
          }
        } else if (++spins >= WIDE_SPIN) {
          st = SETTLED;
          res = -2;
        }
      }
    }
    *slot_out = i;
    return res;
  }
}

// continue an insert from slot i (the slots before it on the probe path are
// held by other states)
__device__ __forceinline__ int fpset_put_from(u64* __restrict__ slots, u64 mask, u64 key, u64 i, u64* slot_out) {
#pragma unroll 1
  for (int p = 0; p < MAX_PROBE; ++p) {
    u64 v = __builtin_nontemporal_load(&slots[i]);
    if (v == key) { *slot_out = i; return 0; }
    if (v == 0) {
      u64 old = atomicCAS((unsigned long long*)&slots[i], 0ull, (unsigned long long)key);
      if (old == 0) { *slot_out = i; return 1; }
      if (old == key) { *slot_out = i; return 0; }
    }
    i = (i + 1) & mask;
  }
  return -1;
}

__device__ __forceinline__ u64 lanemask_lt() {
  const int lane = __lane_id();
  return lane ? (~0ull >> (64 - lane)) : 0ull;
}

// Wave-aggregated append into the block's LDS stage.  Must be reached by all
// lanes of the wave (uniform control flow).
template <bool WITH_SLOT, typename W>
__device__ __forceinline__ void stage_append(bool pred, W st, u64 par, u64 slot, W* s_st, u64* s_par,
                                             u64* s_slot, unsigned* s_cnt) {
  const u64 m = __ballot(pred);
  if (m == 0) return;
  const int leader = __ffsll((long long)m) - 1;
  unsigned base = 0;
  if (__lane_id() == leader) base = atomicAdd(s_cnt, (unsigned)__popcll(m));
  base = __shfl(base, leader);
  if (pred) {
    const unsigned pos = base + (unsigned)__popcll(m & lanemask_lt());
    s_st[pos] = st;
    s_par[pos] = par;
    if (WITH_SLOT) s_slot[pos] = slot;
  }
}

__device__ __forceinline__ u64 wave_sum_u64(u64 v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  return v;
}

// ---- the global engine's check of a new level [g0, g0 + n) when the cfg has
// user invariants (Layout.defer_inv: the expand kernels check none).  Every
// invariant in cfg order on each state; the event key is the state's
// first-discovery key -- its parent reference without the rank, its Init
// index on level 0, or (bit 50) its own store index when its parent lives on
// another rank (tlcgpu.hip resolve_event).  The precompiled k_user_check
// interprets the user program (user_inv.h); the hipRTC build (jit.cpp
// tlcg_user_check) runs it as device code.
struct UserCheckArgs {
  const void* states;
  const u64* parents;
  u64 n;
  int level0;
  unsigned long long* ev;
  u64 rank_tag;  // this rank << 56
  u64 g0;
};

template <typename W>
TLCG_HD u64 user_check_dkey(const Layout& L, const UserCheckArgs& a, u64 i, W s) {
  const u64 pr = a.parents[i];
  return a.level0 ? init_index(L, s)
       : (pr & ~((1ull << 56) - 1)) != a.rank_tag ? (1ull << 50) | (a.g0 + i) : (pr & ((1ull << 56) - 1));
}

#ifdef TLCG_USER_INV
template <typename W>
__device__ __forceinline__ void user_check_body(const UserCheckArgs& a, const Layout& L) {
  const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.n) return;
  const W s = ((const W*)a.states)[i];
  int c = -1;
  for (int q = 0; q < L.n_inv && c < 0; ++q) {
    const int kind = L.inv[q];
    const int r = kind >= INV_USER ? tlcg_user_eval(kind - INV_USER, UVWord<W>{L, s}) : eval_invariant(L, kind, s);
    if (r != EV_TRUE) c = (q << 1) | (r == EV_ERROR ? 1 : 0);
  }
  if (c < 0) return;
  atomicMin(a.ev, (unsigned long long)make_event(user_check_dkey(L, a, i, s), (c & 1) ? EVK_INV_ERROR : EVK_VIOLATION,
                                                 c >> 1));
}
#endif

}  // namespace tlcg
