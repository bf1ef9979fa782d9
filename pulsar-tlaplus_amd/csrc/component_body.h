// pulsar-tlaplus_amd/csrc/component_body.h -- device body of the component
// engine (component.h), shared by the precompiled kernel (component.hip) and
// the run-time specialized one (jit.cpp).
#pragma once
#if !defined(__HIPCC_RTC__)
#include "component.h"
#include "component_model.h"
#include "kernels.h"
#endif

namespace tlcg {

// slot of a local key in a T-slot table (multiply-shift, T need not be a power of 2)
template <int T>
__device__ __forceinline__ unsigned slot_of(uint32_t key) {
  return (unsigned)(((unsigned long long)(key * 0x9E3779B1u) * (unsigned)T) >> 32);
}

// on-chip FPSet slots per component: 1.5 x the capacity (load <= 2/3)
#ifndef TLCG_FPSET_NUM  // on-chip FPSet slots = K * NUM / DEN (tuning hook, jit.cpp)
#define TLCG_FPSET_NUM 3
#define TLCG_FPSET_DEN 2
#endif
template <int K>
struct CompShape { static constexpr int T = (K * TLCG_FPSET_NUM / TLCG_FPSET_DEN + 15) / 16 * 16; };

// the BFS of one wave's components; L is the runtime layout (precompiled
// kernel) or a constexpr one (jit.cpp), in which case every field folds.
// OD: also count TLC's outdegree histogram (a.outdeg; ~9 % of the kernel's
// time on G9, so only when asked for, tlcg_opts.outdegree)
template <int K, bool OD = false>
__device__ __forceinline__ void component_body(const CompArgs& a, const Layout& L) {
  constexpr int T = CompShape<K>::T;
  __shared__ uint32_t q[K][64];                   // FIFO of local keys (word >> msgs_bits)
  __shared__ uint8_t h[T][64];                    // FPSet: 1 + queue position, 0 = empty
  __shared__ unsigned lvl_sh[COMP_MAXLV];
  const int lane = threadIdx.x;
  const int mb = L.msg_sh + L.N * L.mw;  // `messages` occupies the low mb bits
  if (lane < COMP_MAXLV) lvl_sh[lane] = 0;
  u64 gen = 0, dist = 0;
  unsigned od0 = 0, od1 = 0, od2 = 0;  // TLC's outdegree histogram: states with 0 / 1 / 2 new successors
  unsigned long long ev = NO_EVENT;
  __syncthreads();
  for (u64 b = blockIdx.x; b * 64 < a.n_comp; b += gridDim.x) {
    const u64 ci = b * 64 + (u64)lane;
    const bool act = ci < a.n_comp;
    // cascade entries carry the levels an earlier pass already counted (bits 40..)
    const u64 entry = act ? (a.list ? a.list[ci] : a.comp0 + ci) : 0;
    const u64 idx0 = entry & ((1ull << 40) - 1);
    const int counted = (int)(entry >> 40);
    // clear this wave's FPSet with 16-B stores across the whole [T][64] array
    for (int i = lane; i < T * 64 / 16; i += 64) reinterpret_cast<uint4*>(&h[0][0])[i] = make_uint4(0, 0, 0, 0);
    const u64 s0 = init_state(L, idx0);
    const u64 msgs = s0 & L.msgs_mask;
    const CompMsgs cmsg = comp_msgs_init(L, s0);  // everything that reads only `messages`
    u64* st = a.store + b * (u64)K * 64 + (u64)lane;
    u64* par = a.parents + b * (u64)K * 64 + (u64)lane;
    const u64 gbase = a.store_base + b * (u64)K * 64 + (u64)lane;
    // wave-uniform bases + 32-bit lane offsets (saddr + voffset stores), and
    // the parent reference of queue position 0 (+ pos << (6 + ord_bits) per position)
    char* const stb = reinterpret_cast<char*>(a.store + b * (u64)K * 64);
    char* const parb = reinterpret_cast<char*>(a.parents + b * (u64)K * 64);
    const u64 pref = a.rank_tag | (gbase << L.ord_bits);
    int head = 0, tail = 0, level = 0, lvl_end = 0, lvl_start = 0;
    bool alive = act, ovf = false;
    u64 lgen = 0;
    unsigned ocnt = 0;  // this component's outdegree histogram, 10 bits per bin
    u64 lev = NO_EVENT;
    if (act) {
      const uint32_t k0 = (uint32_t)(s0 >> mb);
      h[slot_of<T>(k0)][lane] = 1;
      q[0][lane] = k0;
      tail = 1;
      st[0] = s0;
      par[0] = NO_PARENT;
      lgen = 1;
      const int c = check_invariants_k(L, cmsg, k0);
      if (c >= 0) {  // an initial state violates: level field 0 sorts before every expansion
        lev = make_comp_event(0, idx0, 0, 0, (c & 1) ? EVK_INV_ERROR : EVK_VIOLATION, c >> 1);
        alive = false;
      }
    }
    lvl_end = tail;
    // visit one successor whose probe starts at slot `sl` holding `e`: FPSet
    // lookup, insert, invariants (TLC's FPSet.put + check).  Returns the slot
    // it inserted into, or -1.
    auto visit = [&](lkey key, int action, int pos, unsigned sl, unsigned e) -> int {
      for (int p = 0; p < T; ++p) {
        if (e == 0) break;
        if (q[e - 1][lane] == key) return -1;  // seen
        sl = sl + 1 == (unsigned)T ? 0 : sl + 1;
        e = h[sl][lane];
      }
      if (tail >= K) {  // does not fit on chip: cascade
        ovf = true;
        alive = false;
        return -1;
      }
      h[sl][lane] = (uint8_t)(tail + 1);
      q[tail][lane] = key;
#ifndef TLCG_NO_STORE  // (experiment only: measures what the HBM store costs)
      const unsigned off = (unsigned)(tail * 64 + lane) * 8u;
      *reinterpret_cast<u64*>(stb + off) = msgs | ((u64)key << mb);
      *reinterpret_cast<u64*>(parb + off) = (pref + ((u64)pos << (6 + L.ord_bits))) | (u64)ordinal_of(L, action, 0);
#endif
      ++tail;
      const int c = check_invariants_k(L, cmsg, key);
      if (c >= 0) {
        lev = min(lev, make_comp_event(level + 1, idx0, pos, action, (c & 1) ? EVK_INV_ERROR : EVK_VIOLATION, c >> 1));
        alive = false;
      }
      return (int)sl;
    };
    // the state at the queue head lives in a register; the next one is read
    // from LDS while this one expands
    lkey cur = act ? (lkey)(s0 >> mb) : 0;
    while (alive && head < tail) {
      const lkey s = cur;
      const int tail0 = tail;
      const lkey nxt = head + 1 < tail0 ? q[head + 1][lane] : 0;
      int nsucc = 0;
      lkey t = 0;
      int action = 0;
      // compaction.tla:221-226, on the lane's local key.  Per-lane dispatch on
      // compactorState; TLCG_UNIFORM_PHASE (tuning hook) takes a scalar
      // branch when the wave agrees (measured no faster).
      const int ph = k_phase(L, s);
      const int ph0 = __builtin_amdgcn_readfirstlane(ph);
      int r;
#ifdef TLCG_UNIFORM_PHASE
      if (__all(ph == ph0)) r = compactor_step_k(L, cmsg, msgs, s, ph0, &t, &action);
      else r = compactor_step_k(L, cmsg, msgs, s, ph, &t, &action);
#else
      r = compactor_step_k(L, cmsg, msgs, s, ph, &t, &action);
      (void)ph0;
#endif
      if (r == 2) {
        lev = min(lev, make_comp_event(level + 1, idx0, head, action, EVK_ACTION_ERROR, action));
        alive = false;
        break;
      }
      lkey t2 = 0;
      const bool crash = crash_step_k(L, s, &t2) != 0;  // BrokerCrash, compaction.tla:227
      // both successors' first FPSet slots are read together
      const unsigned sl1 = slot_of<T>(t), sl2 = slot_of<T>(t2);
      const unsigned e1 = r == 1 ? h[sl1][lane] : 0;
      unsigned e2 = crash ? h[sl2][lane] : 0;
      lkey first_new = 0;
      if (r == 1) {
        ++nsucc;
        const int ins = visit(t, action, head, sl1, e1);
        if (ins >= 0) first_new = t;
        if (ins == (int)sl2 && crash) e2 = h[sl2][lane];  // the slot just taken
      }
      if (alive && crash) {
        ++nsucc;
        const int ins = visit(t2, ACT_CRASH, head, sl2, e2);
        if (ins >= 0 && tail0 == tail - 1) first_new = t2;
      }
      nsucc += selfloop_count_k(L, cmsg, s);  // Consumer / Terminating stutters
      lgen += (u64)nsucc;
      if constexpr (OD) ocnt += 1u << (10 * (tail - tail0));  // new states this expansion discovered (0..2)
      if (alive && nsucc == 0 && L.check_deadlock) {
        lev = min(lev, make_comp_event(level + 1, idx0, head, 15, EVK_DEADLOCK, 0));
        alive = false;
      }
      if (!alive) break;
      ++head;
      cur = head < tail0 ? nxt : first_new;  // position head was filled by this expansion
      if (head == lvl_end) {  // level `level` = [lvl_start, lvl_end) is complete
        if (level >= counted) atomicAdd(&lvl_sh[level], (unsigned)(lvl_end - lvl_start));
        ++level;
        if (level >= COMP_MAXLV) {
          ovf = true;
          break;
        }
        lvl_start = head;  // the new level is [head, tail)
        lvl_end = tail;
      }
    }
    if (act && ovf) {
      // the next pass redoes the component and counts only levels >= `level`
      // (the complete ones were counted here, at their transitions)
      const unsigned long long k = atomicAdd(a.ovf_n, 1ull);
      a.ovf_list[k] = idx0 | ((u64)(level > counted ? level : counted) << 40);
    } else if (act) {
      gen += lgen;
      dist += (u64)tail;
      if constexpr (OD) {
        od0 += ocnt & 1023;
        od1 += (ocnt >> 10) & 1023;
        od2 += ocnt >> 20;
      }
      ev = min(ev, (unsigned long long)lev);
      // a lane stopped by an error: `level` = [lvl_start, lvl_end) is partly
      // expanded and level+1 = [lvl_end, tail) partly discovered
      if (lev != NO_EVENT) {
        if (level < COMP_MAXLV && level >= counted) atomicAdd(&lvl_sh[level], (unsigned)(lvl_end - lvl_start));
        if (level + 1 < COMP_MAXLV && level + 1 >= counted && tail > lvl_end)
          atomicAdd(&lvl_sh[level + 1], (unsigned)(tail - lvl_end));
      }
    }
  }
  gen = wave_sum_u64(gen);
  dist = wave_sum_u64(dist);
  const u64 o0 = wave_sum_u64(od0), o1 = wave_sum_u64(od1), o2 = wave_sum_u64(od2);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) ev = min(ev, (unsigned long long)__shfl_xor(ev, off));
  __syncthreads();
  if (lane == 0) {
    if (gen) atomicAdd(&a.totals[0], (unsigned long long)gen);
    if (dist) atomicAdd(&a.totals[1], (unsigned long long)dist);
    if (ev != NO_EVENT) atomicMin(a.event, ev);
    if constexpr (OD) {
      if (o0) atomicAdd(&a.outdeg[0], (unsigned long long)o0);
      if (o1) atomicAdd(&a.outdeg[1], (unsigned long long)o1);
      if (o2) atomicAdd(&a.outdeg[2], (unsigned long long)o2);
    }
  }
  if (lane < COMP_MAXLV && lvl_sh[lane]) atomicAdd(&a.lvl[lane], (unsigned long long)lvl_sh[lane]);
}


}  // namespace tlcg
