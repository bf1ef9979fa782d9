// pulsar-tlaplus_amd/csrc/expand_fast.h -- the global engine's fast BFS
// level (k_expand_fast in tlcgpu.hip, with the runtime layout; jit.cpp
// tlcg_expand_fast_* with the layout a constexpr, so every field folds and
// the kernel's scalar registers no longer hold a Layout: round 6).
#pragma once
#if !defined(__HIPCC_RTC__)
#include "kernels.h"
#include "model.h"
#endif

namespace tlcg {

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
  // a pipelined partition level (ctx_absorb_expand, k_expand_fast_part only):
  // the frontier's size is the preceding absorb's count *n_front_dev (n_front
  // only bounds the grid), states_out / parents_out / cap_out describe the
  // store from the frontier's start (the new states follow the frontier), and
  // a set *guard (that absorb overflowed) makes the launch a no-op
  const unsigned long long* n_front_dev;
  const unsigned* guard;
};

// ---- the fast path of one BFS level (no Producer, discovery order not kept,
// successors stay on this rank): every thread takes IT parents, derives all
// their candidate successors first, then issues the FPSet probes of all of
// them together (2*IT independent loads / CASes in flight per lane) before
// staging the new ones.  PROBE 0: load, CAS only on an empty slot; PROBE 1:
// CAS straight away (one round trip, an atomic on every probe).
template <int IT, int PROBE>
__device__ __forceinline__ void expand_fast_body(const ExpandArgs& a, const Layout& L) {
  constexpr int NC = 2 * IT;
  constexpr int CAP = BLOCK * NC;
  __shared__ u64 s_st[CAP];
  __shared__ u64 s_par[CAP];
  __shared__ unsigned s_cnt;
  __shared__ unsigned long long s_base;
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

}  // namespace tlcg
