// pulsar-tlaplus_amd/csrc/component_wave.h -- the component engine's first
// pass with one walk of the code graph per wavefront (round 5).
//
// component_body.h gives each lane its own FIFO and FPSet in LDS (13.3 KB per
// 64-lane workgroup: 3 waves per SIMD) and has every lane run the same
// transitions on its own registers.  But the successor of a component code
// (component_code.h compactor_step_cb, crash_step_c, selfloop_count_c) reads
// nothing of the component except Len(messages): components with the same
// Len and the same initial code walk the same code graph, visit the same codes
// in the same FIFO order and store the same record at the same queue position.
// So here a wave walks it once for WAVE_M x 64 components (WAVE_M per lane):
//   - the FIFO of codes and the FPSet (1-byte queue positions, the tuned
//     multiply-shift slots) are shared by the wave in LDS (about 0.5 KB per
//     wave), read at wave-uniform addresses; the walk's control -- the loop,
//     the probes, the level transitions -- is scalar, its arithmetic vector
//     (the same value in every lane: the SIMDs issue twice what the CU's one
//     scalar unit does);
//   - the walk's 32-bit records (comp_record: code, parent position, action)
//     are the same for every component of the walk, so they are stored once
//     per walk and queue position (a table of K records per wave iteration,
//     walk = batch / M); a component's slot (batch, position, lane) keeps its
//     numbering and decodes through its walk's record (tlcgpu.hip
//     crec_index, comp_slot_decode) -- the store traffic of one record per
//     component and state (4 B, 0.43 of HBM peak at 1.21 ms for G9) is gone;
//   - each component still gets every one of its states checked against every
//     invariant of the cfg (the spec's own on its component's constants, the
//     user's through their outcome tables), its own event key (TLC's first
//     error of its component) and its own counts, and it stops at the end of
//     the level where it found an error while the others go on.
// Which components share the walk is checked, not assumed: a component joins
// it when its initial local key round-trips through the code, its initial
// code equals the wave leader's and its Len equals the leader's; any other
// goes on to the 32-bit cascade pass (as a component past the pass's capacity
// does).  The level counts of the components in the walk are one add per
// level, not 64 same-address LDS adds (the bank conflicts of component_body.h).
#pragma once
#if !defined(__HIPCC_RTC__)
#include "component_body.h"
#endif

namespace tlcg {

#ifndef TLCG_WAVE_M  // components per lane (component.h WAVE_M; jit.cpp sets it with the module)
#ifdef TLCG_USER_INV
#define TLCG_WAVE_M WAVE_M_USER
#else
#define TLCG_WAVE_M WAVE_M
#endif
#endif

__device__ __forceinline__ uint32_t uni(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }
// a wave-uniform value copied into a vector register: the walk's arithmetic
// on it is issued to the SIMDs rather than to the CU's one scalar unit
__device__ __forceinline__ uint32_t vcopy(uint32_t x) {
  uint32_t v;
  asm volatile("v_mov_b32 %0, %1" : "=v"(v) : "s"(x));
  return v;
}

template <int K, bool OD = false>
__device__ __forceinline__ void component_wave_body(const CompArgs& a, const Layout& L) {
  constexpr int M = TLCG_WAVE_M;
  constexpr int T = CodeShape<K>::T;
  constexpr int LV = TLCG_CODE_MAXLV < COMP_MAXLV ? TLCG_CODE_MAXLV : COMP_MAXLV;  // levels tracked
  __shared__ uint16_t q[K];                  // the wave's FIFO of codes
  // its FPSet: the code + 1, 0 = empty (a probe is one LDS read instead of a
  // queue position and then its queue entry; within 1 %, r05_probe_wave_hkey.jsonl)
  __shared__ uint32_t h[T];
  __shared__ unsigned long long lvl_sh[LV];  // per level: distinct (low 32) + generated (high 32)
  const int lane = threadIdx.x;
  const int mb = L.msg_sh + L.N * L.mw;
  if (lane < LV) lvl_sh[lane] = 0;
  u64 gen = 0, dist = 0;
  u64 wexp = 0;  // the walks' code-state expansions (each once for all the walk's components)
  unsigned od0 = 0, od1 = 0, od2 = 0;
  unsigned long long ev = NO_EVENT;
  // (wave w walks batches w*M .. w*M+M-1; component (batch bm, lane) as in component_body.h)
  for (u64 b0 = (u64)blockIdx.x * M; b0 * 64 < a.n_comp; b0 += (u64)gridDim.x * M) {
    for (int i = lane; i < T; i += 64) h[i] = 0;
    // component m's initial-state index (kept in no register: recomputed)
    auto idx0 = [&](int m) -> u64 {
      const u64 ci = (b0 + m) * 64 + (u64)lane;
      return ci < a.n_comp ? (a.list ? a.list[ci] : a.comp0 + ci) & ((1ull << 40) - 1) : 0;  // (a first pass)
    };
    CodeConsts ccon[M];
#ifndef TLCG_USER_INV
    // past the start, a component of the walk keeps only the flags of its
    // constants (its Len is the walk's): one register instead of a CodeConsts
    uint32_t kf[M];
#endif
    ckey c0[M];
    bool code_ok[M];
    u64 okm = 0;
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const u64 ci = (b0 + m) * 64 + (u64)lane;
      const bool act = ci < a.n_comp;
      const u64 s0 = init_state(L, idx0(m));
      ccon[m] = code_consts(L, comp_msgs_init(L, s0));
#ifdef TLCG_USER_INV
      code_consts_user(L, ccon[m]);  // the user invariants' outcome tables of this component
#endif
      const lkey k0 = (lkey)(s0 >> mb);
      c0[m] = code_encode(L, k0);
      code_ok[m] = act && code_decode(L, ccon[m], c0[m]) == k0;
#ifndef TLCG_USER_INV
      kf[m] = (uint32_t)(ccon[m].msgs_ok != 0) | (uint32_t)(ccon[m].hz_live != 0) << 1 |
              (uint32_t)(ccon[m].hz_false != 0) << 2 | (uint32_t)(ccon[m].dn0 != 0) << 3 | (uint32_t)(ccon[m].dn1 != 0) << 4;
#endif
      okm |= __ballot(code_ok[m]);
    }
    // the walk's leader: the first component of batch 0..M-1 with a code
    int lm = 0;
    u64 lmask = __ballot(code_ok[0]);
#pragma unroll
    for (int m = 1; m < M; ++m)
      if (!lmask) {
        lmask = __ballot(code_ok[m]);
        lm = m;
      }
    const int leader = lmask ? __ffsll((long long)lmask) - 1 : 0;
    ckey lc = c0[0];
    uint32_t ll = ccon[0].len;
#pragma unroll
    for (int m = 1; m < M; ++m)
      if (lm == m) {
        lc = c0[m];
        ll = ccon[m].len;
      }
    const ckey cu0 = (ckey)__builtin_amdgcn_readlane((int)lc, leader);
    const uint32_t lenu = (uint32_t)__builtin_amdgcn_readlane((int)ll, leader);
    // the components of the walk; the others (another code graph, or no code) go on to the cascade
    // (an event key goes to `ev` when found: a component that later leaves for
    // the cascade finds the same key again there)
    // (per component: bit m of a vector register -- as bool arrays they are
    // lane masks in scalar registers, 2 per component and flag, which at M = 10
    // spill; profiles/r05_probe_wave_bits.jsonl)
    uint32_t runb = 0, stopb = 0;
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const bool act = (b0 + m) * 64 + (u64)lane < a.n_comp;
#ifndef TLCG_WAVE_REFUSE_ODD
      const bool r = code_ok[m] && c0[m] == cu0 && ccon[m].len == lenu;
#else
      // (test hook: the components of odd batch + lane parity refuse the walk,
      // so the fallback below and the cascade pass run; tests/test_gpu_wave_parity.py)
      const bool r = code_ok[m] && c0[m] == cu0 && ccon[m].len == lenu && (((b0 + (u64)m) ^ (u64)lane) & 1) == 0;
#endif
      runb |= (uint32_t)r << m;
      if (act && !r) a.ovf_list[atomicAdd(a.ovf_n, 1ull)] = idx0(m);
    }
    auto run = [&](int m) -> bool { return (runb >> m) & 1u; };
    CodeConsts cu{};  // the transitions read Len only
    cu.len = lenu;
    // component m's constants for its invariants (a component of the walk has the walk's Len)
    auto kc = [&](int m) -> CodeConsts {
#ifdef TLCG_USER_INV
      return ccon[m];
#else
      CodeConsts k{};
      k.len = lenu;
      k.msgs_ok = kf[m] & 1;
      k.hz_live = (kf[m] >> 1) & 1;
      k.hz_false = (kf[m] >> 2) & 1;
      k.dn0 = (kf[m] >> 3) & 1;
      k.dn1 = (kf[m] >> 4) & 1;
      return k;
#endif
    };
    __syncthreads();  // (the cleared table)
    if (!okm) continue;
    if (lane == 0) {
      h[slot_of<T>(cu0, a.mult)] = cu0 + 1u;
      q[0] = (uint16_t)cu0;
    }
    u64 lgen = 0;  // successors generated up to the last complete level (the same for every running component)
    unsigned ocnt = 0;
    int n0 = 0;    // components of the walk whose initial state violates
    // the walk's records (range-checked raw buffer stores from lane 0: one per queue position)
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<uint32_t*>(a.store) + (b0 / M) * (u64)K, (short)0, K * 4, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b32(comp_record(cu0, 0, 0), rsrc, lane == 0 ? 0 : 0x7fffffff, 0, 0);
#pragma unroll
    for (int m = 0; m < M; ++m) {
      if (run(m)) {
        const int c = check_invariants_direct(L, kc(m), cu0);
        if (c >= 0) {  // an initial state violates: level 0 is complete, nothing is expanded
          ev = min(ev, (unsigned long long)make_comp_event(0, idx0(m), 0, 0, (c & 1) ? EVK_INV_ERROR : EVK_VIOLATION, c >> 1));
          runb &= ~(1u << m);
          gen += 1;
          dist += 1;
          ++n0;
        }
      }
    }
    lgen = 1;
    {  // those components' level 0 (the others count it when it is expanded)
      const int n = (int)uni((uint32_t)wave_sum_u64((u64)n0));
      if (lane == 0 && n) lvl_sh[0] += (unsigned long long)n;
    }
    __syncthreads();
    auto any_run = [&]() -> bool { return __ballot(runb != 0) != 0; };
    auto n_run = [&]() -> int { return (int)uni((uint32_t)wave_sum_u64((u64)__popc(runb))); };
    int head = 0, tail = 1, level = 0, lvl_start = 0, lvl_end = 1;  // the walk's (scalar)
    unsigned lvgen = 0;
    uint32_t cur = vcopy(cu0);  // the walk's data: vector registers, the same in every lane
    while (any_run()) {
      const uint32_t s = cur;
      const int tail0 = tail;
      ckey t = 0, t2 = 0;
      int action = 0;
      const uint32_t nxt = q[head + 1 < K ? head + 1 : K - 1];
      const int r = (int)uni((uint32_t)compactor_step_cb(L, cu, s, &t, &action));  // compaction.tla:221-226
      const bool crash = uni((uint32_t)crash_step_c(L, s, &t2)) != 0;             // :227
      action = (int)uni((uint32_t)action);
      int nsucc = 0;
      uint32_t first_new = 0;
      // bit m: component m's inserted successor (the compactor's, BrokerCrash's)
      // may violate (its outcome is worked out again in the rare branch: one
      // register each instead of one per component)
      uint32_t evb1 = 0, evb2 = 0;
      // FPSet.put of one successor: a probe of the shared table, and on a miss
      // the insert (the queue; each component's record and invariants).
      // Returns whether it inserted (wave-uniform: the walk's control stays scalar)
      auto put = [&](uint32_t key, int act_id, uint32_t* evb) -> bool {
        unsigned sl = slot_of<T>(key, a.mult);
        unsigned e = h[sl];
        for (int p = 0; uni(e) != 0 && p < T; ++p) {
          if (uni(e == key + 1u ? 1u : 0u)) return false;  // seen
          sl = sl + 1 == (unsigned)T ? 0 : sl + 1;
          e = h[sl];
        }
        // (every lane writes the same word: no exec-mask switch)
        h[sl] = key + 1u;
        q[tail] = (uint16_t)key;
        // the walk's record of position tail (lane 0), then each running
        // component's invariants, with no branch per component: a component
        // out of the walk has its outcome masked
        __builtin_amdgcn_raw_buffer_store_b32(comp_record(key, head, act_id), rsrc, lane == 0 ? tail * 4 : 0x7fffffff, 0, 0);
        uint32_t b = 0;
#ifdef TLCG_USER_INV
#pragma unroll
        for (int m = 0; m < M; ++m) b |= (uint32_t)(check_invariants_cbt(L, kc(m), key) != -1) << m;
#else
        {
          // the spec's invariants read, besides the code and the walk's Len,
          // a component's five flags (kf): lane l evaluates them for the flags
          // l % 32, one ballot gives the outcome of every combination, and
          // each component reads its own bit -- one evaluation per insert
          // instead of one per component
          CodeConsts kl{};
          kl.len = lenu;
          kl.msgs_ok = lane & 1;
          kl.hz_live = (lane >> 1) & 1;
          kl.hz_false = (lane >> 2) & 1;
          kl.dn0 = (lane >> 3) & 1;
          kl.dn1 = (lane >> 4) & 1;
          const uint32_t vf = (uint32_t)__ballot(check_invariants_cbt(L, kl, key) != -1);
#pragma unroll
          for (int m = 0; m < M; ++m) b |= ((vf >> (kf[m] & 31u)) & 1u) << m;
        }
#endif
        *evb = b & runb;
        ++tail;
        __syncthreads();  // (the shared queue and table written)
        return true;
      };
      if (r == 1) {
        ++nsucc;
        if (put(t, action, &evb1)) first_new = t;
      }
      if (crash) {
        ++nsucc;
        if (put(t2, ACT_CRASH, &evb2) && tail0 == tail - 1) first_new = t2;
      }
      nsucc += (int)uni((uint32_t)selfloop_count_c(L, cu, s));  // Consumer / Terminating stutters
      lvgen += (unsigned)nsucc;
      if constexpr (OD) ocnt += 1u << (10 * (tail - tail0));
      // each component's events: an action error, a deadlock (both the
      // walk's), an invariant of an inserted successor (its own); the rare branch
      const bool walk_ev = (r == 2) | (nsucc == 0 && L.check_deadlock);
      const uint32_t evm = (walk_ev ? runb : 0u) | evb1 | evb2;  // components with an event
      if (evm) {
#pragma unroll
      for (int m = 0; m < M; ++m) {
        if ((evm >> m) & 1u) {
          // the successors' outcomes, evaluated on the programs (exact, also
          // where an outcome table left it to them)
          const int ev1 = (evb1 >> m) & 1u ? check_invariants_direct(L, kc(m), t) + 1 : 0;
          const int ev2 = (evb2 >> m) & 1u ? check_invariants_direct(L, kc(m), t2) + 1 : 0;
          u64 k = r == 2 ? make_comp_event(level + 1, idx0(m), head, action, EVK_ACTION_ERROR, action)
                  : nsucc == 0 && L.check_deadlock ? make_comp_event(level + 1, idx0(m), head, 15, EVK_DEADLOCK, 0)
                                                   : NO_EVENT;
          if (ev1)
            k = min(k, make_comp_event(level + 1, idx0(m), head, action, ((ev1 - 1) & 1) ? EVK_INV_ERROR : EVK_VIOLATION,
                                       (ev1 - 1) >> 1));
          if (ev2)
            k = min(k, make_comp_event(level + 1, idx0(m), head, ACT_CRASH,
                                       ((ev2 - 1) & 1) ? EVK_INV_ERROR : EVK_VIOLATION, (ev2 - 1) >> 1));
          ev = min(ev, (unsigned long long)k);
          stopb |= (uint32_t)(k != NO_EVENT) << m;
        }
      }
      }
      ++head;
      cur = head < tail0 ? nxt : first_new;  // position head was filled by this expansion
      const bool done = head >= tail;        // the component ran out (every component of the walk)
      bool deep = false, ended = false;
      if (head == lvl_end) {  // level `level` = [lvl_start, lvl_end) is complete and expanded
        const int n = n_run();
        if (lane == 0 && n)
          lvl_sh[level] += (unsigned long long)((lvl_end - lvl_start) * n) | ((unsigned long long)lvgen * (unsigned)n << 32);
        lgen += lvgen;
        lvgen = 0;
        ++level;
        lvl_start = head;  // the new level is [head, tail)
        lvl_end = tail;
        deep = level >= LV;  // more levels than tracked on chip: the cascade
        ended = true;
      }
      // leaving: an error in the level just expanded (the new level is not
      // expanded) or the component ran out -- its counts complete -- or, to
      // the cascade, too deep or no room for the next expansion's two
      // successors (component_body.h's order of these tests)
      int nq = 0;
      if (ended || done || tail > K - 2)  // (the walk's conditions: most expansions skip this)
#pragma unroll
      for (int m = 0; m < M; ++m) {
        const bool quit = run(m) && !deep && ((ended && ((stopb >> m) & 1u)) || done);
        const bool ovf = run(m) && !quit && (deep || tail > K - 2);
        if (ovf) a.ovf_list[atomicAdd(a.ovf_n, 1ull)] = idx0(m) | ((u64)level << 40);  // levels < `level` counted
        if (quit) {
          // the last level [lvl_start, tail) was discovered, not expanded
          gen += lgen;
          dist += (u64)tail;
          if constexpr (OD) {
            od0 += ocnt & 1023;
            od1 += (ocnt >> 10) & 1023;
            od2 += ocnt >> 20;
          }
          ++nq;
        }
        if (ovf || quit) runb &= ~(1u << m);
      }
      const int nqw = (int)uni((uint32_t)wave_sum_u64((u64)nq));
      if (lane == 0 && nqw && tail > lvl_start) lvl_sh[level] += (unsigned long long)((tail - lvl_start) * nqw);
    }
    wexp += (u64)head;  // (scalar: the walk's expanded code states)
    __syncthreads();  // (the next batches clear the table)
  }
  gen = wave_sum_u64(gen);
  dist = wave_sum_u64(dist);
  const u64 o0 = wave_sum_u64(od0), o1 = wave_sum_u64(od1), o2 = wave_sum_u64(od2);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) ev = min(ev, (unsigned long long)__shfl_xor(ev, off));
  __syncthreads();
  const u64 so = a.nstripe > 1 ? (u64)(blockIdx.x % (unsigned)a.nstripe) * a.stripe : 0;  // this workgroup's copy
  if (lane == 0) {
    if (wexp && a.expansions) atomicAdd(&a.expansions[so], (unsigned long long)wexp);
    if (gen) atomicAdd(&a.totals[so + 0], (unsigned long long)gen);
    if (dist) atomicAdd(&a.totals[so + 1], (unsigned long long)dist);
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
