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
enum Overflow { OVF_FPSET = 1, OVF_STORE = 2, OVF_OUTBOX = 4, OVF_DUP_INIT = 8 };

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
__device__ __forceinline__ int fpset_put(u64* __restrict__ slots, int log2, u64 state, u64 fp,
                                         u64* slot_out) {
  const u64 key = state | SLOT_TAG;
  const u64 mask = (1ull << log2) - 1;
  u64 i = fp >> (64 - log2);
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
template <bool WITH_SLOT>
__device__ __forceinline__ void stage_append(bool pred, u64 st, u64 par, u64 slot, u64* s_st, u64* s_par,
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

// arguments of one BFS level's expansion (the global engine)
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

__device__ __forceinline__ u64 wave_sum_u64(u64 v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  return v;
}

}  // namespace tlcg
