// pulsar-tlaplus_amd/csrc/component_lane.h -- the component engine's per-lane
// code pass with a bitmap FPSet and wave-uniform control (round 6).
//
// Like component_body.h, every lane runs TLC's FIFO BFS on its own component
// (compaction.tla:216-231): it expands each of its states (the compactor
// disjunct, BrokerCrash, the stutters), probes and inserts each successor in
// its own FPSet, evaluates every invariant of the cfg on each new state
// (:236-294) and stores each new state's 32-bit record (comp_record).  What
// changes is how a lane's FPSet and FIFO are laid out:
//
//   - FPSet: without a Producer every component walks the same code graph
//     (component_code.h), so the host finds a multiply-shift slot hash that is
//     injective on component 0's code set S (build_lane_phash, host_model.h:
//     T = 256 slots, the top 8 bits of code x a 24-bit multiplier), and a
//     workgroup-shared table owner[slot] = the code of S in that slot + 1.
//     A lane's FPSet is then one bit per slot (T / 32 LDS dwords in lane
//     columns: the lane's own bank, no conflicts), and FPSet.put of code c is
//     exact for any c: c is in the set iff owner[slot(c)] = c + 1 and the
//     lane's bit is set; a successor outside S (owner[slot(c)] != c + 1) means
//     this component's code graph is not S, and the component goes on to the
//     32-bit cascade pass, as one past the pass's capacity does.  A probe is
//     two independent LDS reads (the shared owner word, the lane's bit word)
//     instead of a slot read and then its queue entry, and an insert is two
//     LDS writes.
//   - FIFO: the FPSet no longer points into the queue, so a lane keeps only
//     its unexpanded states, in a ring of LANE_R codes (lane columns); queue
//     positions are counters (the records' numbering is component_body.h's).
//   - control: the BFS loop runs while any lane of the wave is alive, with
//     every lane in it (a finished lane's updates are masked by selects, its
//     record stores go out of the buffer's range), so the per-level counts of
//     the lanes that close a level at one level are one DPP sum and one LDS
//     add instead of 64 same-address LDS adds (component_body.h's bank
//     conflicts), and the loop pays no exec-mask bookkeeping per branch.
// LDS per 64-lane workgroup: the ring R x 128 B (the host picks R per layout,
// jit.cpp / host_model.cpp lane_ring_entries: 8 entries, 1 KB, on G9; a wider
// frontier sends the component to the cascade), the bits 2 KB, owner 1 KB (vs
// 13.3 KB for component_body.h), so registers, not LDS, set the occupancy.
#pragma once
#if !defined(__HIPCC_RTC__)
#include "component_body.h"
#endif

namespace tlcg {

#ifndef TLCG_LANE_R
#define TLCG_LANE_R 16
#endif
constexpr int LANE_R = TLCG_LANE_R;  // FIFO ring entries per lane (a power of 2; the hipRTC module defines it)
// the compactor disjunct through its update masks (component_code.h
// compactor_step_tab: one LDS read and a few bit operations instead of the six
// candidate successors of compactor_step_cb); 0: compactor_step_cb (A/B)
#ifndef TLCG_LANE_STEP_TAB
#define TLCG_LANE_STEP_TAB 1
#endif

// the sum over the wave of x (every lane active), in a scalar
__device__ __forceinline__ uint32_t lane_wave_sum(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, true);  // row_shr:1
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, true);  // row_shr:2
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, true);  // row_shr:4
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, true);  // row_shr:8
  return (uint32_t)__builtin_amdgcn_readlane((int)x, 15) + (uint32_t)__builtin_amdgcn_readlane((int)x, 31) +
         (uint32_t)__builtin_amdgcn_readlane((int)x, 47) + (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
}

template <int K, bool OD = false>
__device__ __forceinline__ void component_lane_body(const CompArgs& a, const Layout& L) {
  static_assert(K <= 64, "records and the 16-bit level sums take K <= 64");
  constexpr int T = LANE_T, NW = T / 32, R = LANE_R;
  constexpr int LV = TLCG_CODE_MAXLV < COMP_MAXLV ? TLCG_CODE_MAXLV : COMP_MAXLV;  // levels tracked
  __shared__ uint16_t ring[R][64];             // the lanes' FIFOs (unexpanded codes)
  __shared__ uint32_t bits[NW][64];            // the lanes' FPSets: bit s of lane l = bit s % 32 of bits[s / 32][l]
  __shared__ uint32_t owner[T];                // the code in slot s + 1 (0: none), shared
  __shared__ unsigned long long lvl_sh[LV];    // per level: distinct (low 32) + generated (high 32)
#if TLCG_LANE_STEP_TAB
  __shared__ u64 steps[STEP_TAB];              // the compactor disjunct's update masks (compactor_step_entry)
#endif
  const int lane = threadIdx.x;
  const int mb = L.msg_sh + L.N * L.mw;
  const uint32_t mult = a.lane_mult;
  for (int i = lane; i < T; i += 64) owner[i] = a.lane_owner[i];
#if TLCG_LANE_STEP_TAB
  for (int i = lane; i < STEP_TAB; i += 64) steps[i] = compactor_step_entry(L, i);
#endif
  if (lane < LV) lvl_sh[lane] = 0;
  uint32_t gen = 0, dist = 0, nexp = 0;  // (nexp: states expanded by the components that finish here)
  unsigned od0 = 0, od1 = 0, od2 = 0;
  unsigned long long ev = NO_EVENT;
  __syncthreads();
  // a level's per-lane counts (x: distinct | generated << 16) into lvl_sh:
  // one DPP sum when every lane that adds adds at one level, else per lane
  auto level_add = [&](bool add, int lvc, uint32_t x) {
    const unsigned long long m = __ballot(add);
    if (!m) return;
    const int l0 = __builtin_amdgcn_readlane(lvc, __ffsll((long long)m) - 1);
    if (!__ballot(add && lvc != l0)) {
      const uint32_t s = lane_wave_sum(add ? x : 0u);
      if (lane == 0) atomicAdd(&lvl_sh[l0], (unsigned long long)(s & 0xFFFFu) | ((unsigned long long)(s >> 16) << 32));
    } else if (add) {
      atomicAdd(&lvl_sh[lvc], (unsigned long long)(x & 0xFFFFu) | ((unsigned long long)(x >> 16) << 32));
    }
  };
  for (u64 b = blockIdx.x; b * 64 < a.n_comp; b += gridDim.x) {
    const u64 ci = b * 64 + (u64)lane;
    const bool act = ci < a.n_comp;
    // cascade entries carry the levels an earlier pass already counted (bits 40..)
    const u64 entry = act ? (a.list ? a.list[ci] : a.comp0 + ci) : 0;
    const u64 idx0 = entry & ((1ull << 40) - 1);
    const int counted = (int)(entry >> 40);
#pragma unroll
    for (int i = 0; i < NW; ++i) bits[i][lane] = 0u;  // (the lane's own columns)
    const u64 s0 = init_state(L, idx0);
    CodeConsts ccon = code_consts(L, comp_msgs_init(L, s0));
#ifdef TLCG_USER_INV
    code_consts_user(L, ccon);  // the user invariants' outcome tables of this component
#endif
    // the records of this batch: [K][64] 32-bit words, position p of lane l at
    // (p x 64 + l) x 4; a store at an offset past the range is dropped
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<uint32_t*>(a.store) + b * (u64)K * 64, (short)0, K * 64 * 4, 0x00020000);
    constexpr int OOB = 0x7fffffff;
    const unsigned loff = (unsigned)lane * 4u;
    int head = 0, tail = 0, level = 0, lvl_start = 0, lvl_end = 0;
    // alive: the BFS goes on; stop: an error was found, so the lane finishes
    // the current level and stops at its end (end-of-level counts, as every
    // engine reports them); ovf: the component goes on to the cascade
    bool alive = act, ovf = false, stop = false;
    uint32_t lgen = 0, lvgen = 0, ocnt = 0;
    u64 lev = NO_EVENT;
    const lkey k0 = act ? (lkey)(s0 >> mb) : 0;
    const ckey c0 = code_encode(L, k0);
    const unsigned p0 = lane_slot(c0, mult);
    if (act && (code_decode(L, ccon, c0) != k0 || owner[p0] != c0 + 1u)) {
      // no code, or not the code graph the slots were built for: the cascade
      ovf = true;
      alive = false;
    }
    if (alive) {
      bits[p0 >> 5][lane] = 1u << (p0 & 31);
      ring[0][lane] = (uint16_t)c0;
      tail = 1;
      __builtin_amdgcn_raw_buffer_store_b32(comp_record(c0, 0, 0), rsrc, (int)loff, 0, 0);  // (position 0: the root)
      lgen = 1;
      const int c = check_invariants_direct(L, ccon, c0);
      if (c >= 0) {  // an initial state violates: level 0 is complete, nothing is expanded
        lev = make_comp_event(0, idx0, 0, 0, (c & 1) ? EVK_INV_ERROR : EVK_VIOLATION, c >> 1);
        alive = false;
        stop = true;
      }
    }
    lvl_end = tail;
    ckey cur = c0;
    while (__ballot(alive)) {
      const ckey s = cur;
      const int tail0 = tail;
      const ckey nxt = ring[(head + 1) & (R - 1)][lane];
      ckey t = 0, t2 = 0;
      int action = 0;
#if TLCG_LANE_STEP_TAB
      const int r = compactor_step_tab(L, ccon, steps, s, &t, &action);  // compaction.tla:221-226
#else
      const int r = compactor_step_cb(L, ccon, s, &t, &action);
#endif
      const bool crash = crash_step_c(L, s, &t2) != 0;            // :227
      // FPSet.put of both successors: slot, the shared owner, the lane's bits
      const unsigned p1 = lane_slot(t, mult), p2 = lane_slot(t2, mult);
      const uint32_t o1 = owner[p1], o2 = owner[p2];
      const uint32_t w1 = bits[p1 >> 5][lane];
      uint32_t w2 = bits[p2 >> 5][lane];
#ifndef TLCG_LANE_NO_SCHED_BARRIER
      // (the four reads issued together, before anything that consumes them
      // or writes LDS: one round trip per expansion, not two)
      __builtin_amdgcn_sched_barrier(0);
#endif
      const uint32_t b1 = 1u << (p1 & 31), b2 = 1u << (p2 & 31);
      const bool e1 = alive && r == 1, e2 = alive && crash;
      const bool in1 = o1 == t + 1u, in2 = o2 == t2 + 1u;
      // a successor outside the code set: this component is not S's, the cascade
      const bool out = (e1 && !in1) || (e2 && !in2);
      const bool new1 = e1 && in1 && !(w1 & b1) && !out;
      if ((p2 >> 5) == (p1 >> 5) && new1) w2 |= b1;  // (the second sees the first's insert)
      const bool new2 = e2 && in2 && !(w2 & b2) && !out;
      bits[p1 >> 5][lane] = new1 ? w1 | b1 : w1;
      bits[p2 >> 5][lane] = new2 ? w2 | b2 : w2;
      // the queue (the ring: a successor not inserted is overwritten or never
      // read) and each new state's record at its position
      ring[tail & (R - 1)][lane] = (uint16_t)t;
      ring[(tail + (new1 ? 1 : 0)) & (R - 1)][lane] = (uint16_t)t2;
#ifndef TLCG_NO_STORE  // (experiment only: measures what the records cost)
      __builtin_amdgcn_raw_buffer_store_b32(comp_record(t, head, action), rsrc,
                                            new1 ? (int)((unsigned)tail * 256u + loff) : OOB, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b32(comp_record(t2, head, ACT_CRASH), rsrc,
                                            new2 ? (int)((unsigned)(tail + (new1 ? 1 : 0)) * 256u + loff) : OOB, 0,
                                            0);
#endif
      const ckey first_new = new1 ? t : t2;
      tail += (new1 ? 1 : 0) + (new2 ? 1 : 0);
      const int nsucc = (e1 ? 1 : 0) + (e2 ? 1 : 0) + (alive ? selfloop_count_c(L, ccon, s) : 0);  // + stutters
      lvgen += (unsigned)nsucc;
      if constexpr (OD) ocnt += alive ? 1u << (10 * (tail - tail0)) : 0u;  // new states this expansion discovered
      // the inserted successors' invariants (first failing + 1; INV_UNKNOWN
      // + 1: an outcome table left it to the programs, the rare branch)
#if defined(TLCG_LANE_INV_UNCOND) && !defined(TLCG_NO_INV)  // (A/B: both evaluated, no branch)
      const int q1 = check_invariants_cbt(L, ccon, t) + 1, q2 = check_invariants_cbt(L, ccon, t2) + 1;
      int ev1 = new1 ? q1 : 0;
      int ev2 = new2 ? q2 : 0;
#elif !defined(TLCG_NO_INV)  // (TLCG_NO_INV: experiment only, measures what the invariants cost)
      int ev1 = new1 ? check_invariants_cbt(L, ccon, t) + 1 : 0;
      int ev2 = new2 ? check_invariants_cbt(L, ccon, t2) + 1 : 0;
#else
      int ev1 = 0, ev2 = 0;
#endif
      // an action error (no successor from the failing action; the others
      // still count, as k_expand), a deadlock and the successors' invariant
      // events in one rare branch
      const bool rare = alive && ((r == 2) | (nsucc == 0 && L.check_deadlock) | (ev1 != 0) | (ev2 != 0));
      if (__ballot(rare)) {
        if (rare) {
#pragma nounroll
          for (int i = 0; i < 2; ++i) {
            if ((i ? ev2 : ev1) == INV_UNKNOWN + 1) {
              const int e = check_invariants_direct(L, ccon, i ? t2 : t) + 1;
              if (i) ev2 = e;
              else ev1 = e;
            }
          }
          u64 k = r == 2 ? make_comp_event(level + 1, idx0, head, action, EVK_ACTION_ERROR, action)
                  : nsucc == 0 && L.check_deadlock ? make_comp_event(level + 1, idx0, head, 15, EVK_DEADLOCK, 0)
                                                   : NO_EVENT;
          if (ev1) k = min(k, make_comp_event(level + 1, idx0, head, action, ((ev1 - 1) & 1) ? EVK_INV_ERROR : EVK_VIOLATION, (ev1 - 1) >> 1));
          if (ev2) k = min(k, make_comp_event(level + 1, idx0, head, ACT_CRASH, ((ev2 - 1) & 1) ? EVK_INV_ERROR : EVK_VIOLATION, (ev2 - 1) >> 1));
          lev = min(lev, k);
          stop = stop || k != NO_EVENT;  // (no event: every unknown outcome held)
        }
      }
      if (alive) ++head;
      cur = head < tail0 ? nxt : first_new;  // position head was filled by this expansion
      bool brk = alive && head >= tail;      // the component ran out
      // level `level` = [lvl_start, lvl_end) complete and expanded
      const bool ended = alive && head == lvl_end;
      if (__ballot(ended)) {
        const int lvc = level < LV ? level : LV - 1;
        level_add(ended && level >= counted, lvc, (uint32_t)(lvl_end - lvl_start) | (lvgen << 16));
        if (ended) {
          lgen += lvgen;
          lvgen = 0;
          ++level;
          lvl_start = head;  // the new level is [head, tail)
          lvl_end = tail;
          const bool deep = level >= LV;  // more levels than tracked on chip: cascade
          ovf = ovf || deep;
          brk = brk || deep || stop;  // stop: an error in the level just expanded, the new level is not expanded
        }
      }
      // room for both successors of the next expansion, in the records and
      // in the ring (checked once per expansion; a component of K - 1 or K
      // states goes on to the cascade too)
      const bool full = alive && !brk && (tail > K - 2 || tail - head > R - 2);
      ovf = ovf || full || out;
      alive = alive && !(brk || full || out);
    }
    if (act && ovf) {
      // the next pass redoes the component and counts only levels >= `level`
      // (the complete ones were counted here, at their transitions)
      const unsigned long long k = atomicAdd(a.ovf_n, 1ull);
      a.ovf_list[k] = idx0 | ((u64)(level > counted ? level : counted) << 40);
    }
    // the last level [lvl_start, tail) was discovered, not expanded (empty
    // when the component ran out)
    const bool fin = act && !ovf;
    const int lvc = level < LV ? level : LV - 1;
    level_add(fin && tail > lvl_start && level >= counted, lvc, (uint32_t)(tail - lvl_start));
    if (fin) {
      gen += lgen;
      dist += (uint32_t)tail;
      nexp += (uint32_t)head;
      if constexpr (OD) {
        od0 += ocnt & 1023;
        od1 += (ocnt >> 10) & 1023;
        od2 += ocnt >> 20;
      }
      ev = min(ev, (unsigned long long)lev);
    }
  }
  const u64 g64 = wave_sum_u64(gen), d64 = wave_sum_u64(dist), x64 = wave_sum_u64(nexp);
  const u64 o0 = wave_sum_u64(od0), o1 = wave_sum_u64(od1), o2 = wave_sum_u64(od2);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) ev = min(ev, (unsigned long long)__shfl_xor(ev, off));
  __syncthreads();
  const u64 so = a.nstripe > 1 ? (u64)(blockIdx.x % (unsigned)a.nstripe) * a.stripe : 0;  // this workgroup's copy
  if (lane == 0) {
    if (x64 && a.expansions) atomicAdd(&a.expansions[so], (unsigned long long)x64);
    if (g64) atomicAdd(&a.totals[so + 0], (unsigned long long)g64);
    if (d64) atomicAdd(&a.totals[so + 1], (unsigned long long)d64);
    if (ev != NO_EVENT) atomicMin(a.event, ev);
    if constexpr (OD) {
      if (o0) atomicAdd(&a.outdeg[so + 0], (unsigned long long)o0);
      if (o1) atomicAdd(&a.outdeg[so + 1], (unsigned long long)o1);
      if (o2) atomicAdd(&a.outdeg[so + 2], (unsigned long long)o2);
    }
  }
  if (lane < LV && lvl_sh[lane]) {
    atomicAdd(&a.lvl[so + lane], lvl_sh[lane] & 0xffffffffull);
    if (lvl_sh[lane] >> 32) atomicAdd(&a.lvl_gen[so + lane], lvl_sh[lane] >> 32);
  }
}

}  // namespace tlcg
