// pulsar-tlaplus_amd/csrc/tree_wave.h -- the component tree's closed mode
// with one walk of the code graph per wavefront (round 5; component_wave.h
// does the same for the component engine's one-lane components).
//
// tree_body.h's closed mode gives every component a group of 16 lanes and its
// own FPSet: a depth of G9-deep's components holds 7.5 states on average, so
// most lanes idle in each step and every step pays its loop, ballot and
// exec-mask instructions per group (8.8 VALU wave-instructions per state,
// profiles/r04_pmc_tree_g9deep.json).  But a component code's successors
// (component_code.h compactor_step_cb, crash_step_c, selfloop_count_c) read
// nothing of the component except Len(messages): components with one Len and
// one initial code walk the same code graph and put the same code at the
// same queue position.  So here a wave walks it once for up to
// TLCG_TREE_WAVE_M x 64 components (one per lane and batch):
//   - the FIFO of codes and the FPSet (1 + queue position per slot) are the
//     wave's, in LDS, read at wave-uniform addresses; the walk's control is
//     scalar and its arithmetic vector (vcopy, component_wave.h);
//   - the walk's records (code, parent queue position, action) are the same
//     for every component of the walk: they are stored once per walk and
//     position (TreeArgs::walk_rec) and each component names its walk
//     (walk_of); a component's slot (tree_wave_slot) keeps its numbering and
//     decodes through its walk's record (tlcgpu.hip tree_wave_record);
//   - each component still gets every state checked against every invariant
//     of the cfg on its own constants (its `messages`: CodeConsts), its own
//     least error key (tree_event_key) and its size; the per-depth counts are
//     one add per depth for all the components of the walk.
// Components that do not share the leader's code graph (another initial code
// or Len) take the next walk of the same wave; a component without a code
// (its initial state does not round-trip) or past CAP states or TREE_MAXLV
// depths raises TREE_OVERFLOW, as in tree_body.h (the 2048-state pass).
//
// Slot numbering: lane-interleaved -- slot (ci, pos) = ((ci / 64) * CAP +
// pos) * 64 + ci % 64 (tree_wave_slot), the layout in which the first
// version stored every component's code and parent reference (12 B per
// state: 2.62 ms for G9-deep, 0.57 of HBM peak, profiles/r05_bench_g9deep.json).
#pragma once
#if !defined(__HIPCC_RTC__)
#include "component_wave.h"
#include "tree_body.h"
#endif

namespace tlcg {

#ifndef TLCG_TREE_WAVE_M  // batches of 64 components per wave (tree.h TREE_WAVE_M; a tuning hook)
#define TLCG_TREE_WAVE_M TREE_WAVE_M
#endif

TLCG_HD u64 tree_wave_slot(u64 ci, u64 pos, int cap) { return ((ci >> 6) * (u64)cap + pos) * 64 + (ci & 63); }

template <int CAP, typename W>
__device__ __forceinline__ void tree_wave_body(const TreeArgs& a, const Layout& L) {
  constexpr int M = TLCG_TREE_WAVE_M;
  constexpr int T = CAP <= 1024 ? 2048 : 4096;  // FPSet slots (load <= 0.31 at CAP 640)
  constexpr int TB = T == 2048 ? 11 : 12;
  __shared__ uint32_t q[CAP];               // the wave's FIFO of codes
  __shared__ uint32_t h[T];                 // its FPSet: the code + 1, 0 = empty (a probe is one LDS read)
  __shared__ unsigned long long lvl_d[TREE_MAXLV], lvl_g[TREE_MAXLV];
  const int lane = threadIdx.x;
  for (int i = lane; i < TREE_MAXLV; i += 64) lvl_d[i] = lvl_g[i] = 0;
  unsigned flags = 0;
  uint32_t maxn = 0;
  u64 nexp = 0;  // code states the walks expanded (lane-uniform)
  u64 evk = ~0ull;  // this lane's least error key
  const u64 nb = (a.n_comp + 63) / 64;
  const int ord_crash = ordinal_of(L, ACT_CRASH, 0);
  for (u64 b0 = (u64)blockIdx.x * M; b0 < nb; b0 += (u64)gridDim.x * M) {
#ifdef TLCG_USER_INV
    CodeConsts ccon[M];
#else
    // the spec's invariants read, besides the code and the walk's Len, five
    // flags of a component's constants (and its Len: bits 8..): one register
    uint32_t kf[M];
#endif
    ckey c0[M];
    uint32_t todob = 0;  // (per component: bit m of a vector register, not a lane mask in scalar registers)
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const u64 ci = (b0 + m) * 64 + (u64)lane;
      const bool act = ci < a.n_comp;
      const W s0 = init_state<W>(L, a.comp0 + (act ? ci : 0));
      CodeConsts k = code_consts(L, comp_msgs_init(L, (u64)s0));  // (`messages` sits in the low word)
#ifdef TLCG_USER_INV
      code_consts_user<W>(L, k);  // the user invariants' outcome tables of this component
      ccon[m] = k;
#else
      kf[m] = (uint32_t)(k.msgs_ok != 0) | (uint32_t)(k.hz_live != 0) << 1 | (uint32_t)(k.hz_false != 0) << 2 |
              (uint32_t)(k.dn0 != 0) << 3 | (uint32_t)(k.dn1 != 0) << 4 | k.len << 8;
#endif
      c0[m] = code_encode_w<W>(L, s0);
      const bool ok = act && code_word<W>(L, k, s0 & messages_mask<W>(L), c0[m]) == s0;
      todob |= (uint32_t)ok << m;
      if (act && !ok) flags |= TREE_OVERFLOW;  // no code
    }
    auto len_of = [&](int m) -> uint32_t {
#ifdef TLCG_USER_INV
      return ccon[m].len;
#else
      return kf[m] >> 8;
#endif
    };
    for (;;) {
      // the walk's leader: the first component still to walk
      int lm = -1;
      u64 lmask = 0;
#pragma unroll
      for (int m = 0; m < M; ++m)
        if (lm < 0) {
          lmask = __ballot((todob >> m) & 1u);
          if (lmask) lm = m;
        }
      if (lm < 0) break;
      const int leader = __ffsll((long long)lmask) - 1;
      ckey lc = c0[0];
      uint32_t ll = len_of(0);
#pragma unroll
      for (int m = 1; m < M; ++m)
        if (lm == m) {
          lc = c0[m];
          ll = len_of(m);
        }
      const ckey cu0 = (ckey)__builtin_amdgcn_readlane((int)lc, leader);
      const uint32_t lenu = (uint32_t)__builtin_amdgcn_readlane((int)ll, leader);
      uint32_t inb = 0;
#pragma unroll
      for (int m = 0; m < M; ++m) inb |= (uint32_t)(((todob >> m) & 1u) && c0[m] == cu0 && len_of(m) == lenu) << m;
      todob &= ~inb;
      const int nin = __popc(inb);
      auto in = [&](int m) -> bool { return (inb >> m) & 1u; };
      const unsigned nwalk = uni((uint32_t)wave_sum_u64((u64)nin));  // components of this walk
      // the walk's number: its records' row (past walk_cap: the 2048-state pass takes the model)
      unsigned long long wid = 0;
      if (lane == 0) wid = atomicAdd(a.walk_n, 1ull);
      wid = __builtin_amdgcn_readfirstlane((unsigned)wid);
      if (wid >= a.walk_cap) {
        flags |= TREE_OVERFLOW;
        break;
      }
#pragma unroll
      for (int m = 0; m < M; ++m)
        if (in(m)) a.walk_of[(b0 + m) * 64 + (u64)lane] = (uint32_t)wid;
      // its records (range-checked raw buffer stores from lane 0)
      const __amdgpu_buffer_rsrc_t rr =
          __builtin_amdgcn_make_buffer_rsrc(a.walk_rec + wid * (u64)CAP, (short)0, CAP * 8, 0x00020000);
      CodeConsts cu{};  // the transitions read Len only
      cu.len = lenu;
      // bit m: component m's state with code `key` violates an invariant.  The
      // spec's invariants read the code, the walk's Len and five flags of a
      // component (kf): lane l evaluates them for the flags l % 32, one ballot
      // gives every combination's outcome, each component reads its bit
      auto violators = [&](ckey key) -> uint32_t {
        uint32_t b = 0;
#ifdef TLCG_USER_INV
#pragma unroll
        for (int m = 0; m < M; ++m) b |= (uint32_t)(check_invariants_cb<W>(L, ccon[m], key) >= 0) << m;
#else
        CodeConsts kl{};
        kl.len = lenu;
        kl.msgs_ok = lane & 1;
        kl.hz_live = (lane >> 1) & 1;
        kl.hz_false = (lane >> 2) & 1;
        kl.dn0 = (lane >> 3) & 1;
        kl.dn1 = (lane >> 4) & 1;
        const uint32_t vf = (uint32_t)__ballot(check_invariants_cb<W>(L, kl, key) >= 0);
#pragma unroll
        for (int m = 0; m < M; ++m) b |= ((vf >> (kf[m] & 31u)) & 1u) << m;
#endif
        return b & inb;
      };
      for (int i = lane; i < T; i += 64) h[i] = 0;
      __syncthreads();
      if (lane == 0) {
        h[(cu0 * 0x9E3779B1u) >> (32 - TB)] = cu0 + 1u;
        q[0] = cu0;
      }
      // position 0: the initial state (no parent)
      __builtin_amdgcn_raw_buffer_store_b32(cu0, rr, lane == 0 ? 0 : 0x7fffffff, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b32(0u, rr, lane == 0 ? 4 : 0x7fffffff, 0, 0);
      {
        const uint32_t vb = violators(cu0);
        if (vb) evk = min(evk, tree_event_key(0, a.comp0 + (b0 + (u64)(__ffs(vb) - 1)) * 64 + (u64)lane));
      }
      __syncthreads();
      int head = 0, tail = 1, level = 0, lvl_start = 0, lvl_end = 1;  // the walk's (scalar)
      unsigned lvgen = 0;
      bool full = false;  // past CAP states or TREE_MAXLV depths: TREE_OVERFLOW
      uint32_t cur = vcopy(cu0);
      for (;;) {
        const uint32_t s = cur;
        const int tail0 = tail;
        ckey t = 0, t2 = 0;
        int action = 0;
        const uint32_t nxt = q[head + 1 < CAP ? head + 1 : CAP - 1];
        const int r = (int)uni((uint32_t)compactor_step_cb(L, cu, s, &t, &action));  // compaction.tla:221-226
        const bool crash = uni((uint32_t)crash_step_c(L, s, &t2)) != 0;             // :227
        action = (int)uni((uint32_t)action);
        int nsucc = 0;
        uint32_t first_new = 0;
        // FPSet.put of one successor: a probe of the shared table; on a miss
        // the queue, each component's code, parent reference and invariants
        auto put = [&](uint32_t key, int ord) -> bool {
          unsigned sl = (key * 0x9E3779B1u) >> (32 - TB);
          unsigned e = h[sl];
          for (int p = 0; uni(e) != 0 && p < T; ++p) {
            if (uni(e == key + 1u ? 1u : 0u)) return false;  // seen
            sl = (sl + 1) & (T - 1);
            e = h[sl];
          }
          if (tail >= CAP) {  // no room: the component does not fit this pass
            full = true;
            return false;
          }
          h[sl] = key + 1u;
          q[tail] = key;
          // the walk's record of position tail: code, parent position, parent ordinal
          __builtin_amdgcn_raw_buffer_store_b32(key, rr, lane == 0 ? tail * 8 : 0x7fffffff, 0, 0);
          __builtin_amdgcn_raw_buffer_store_b32((uint32_t)head | (uint32_t)ord << 16, rr, lane == 0 ? tail * 8 + 4 : 0x7fffffff,
                                                0, 0);
          // each component's invariants: a bit per violating component; its
          // key (the least is the first component's) only in the rare branch
          const uint32_t vb = violators(key);
          if (vb) evk = min(evk, tree_event_key(level + 1, a.comp0 + (b0 + (u64)(__ffs(vb) - 1)) * 64 + (u64)lane));
          ++tail;
          __syncthreads();  // (the shared queue and table written)
          return true;
        };
        if (r == 1) {
          ++nsucc;
          if (put(t, ordinal_of(L, action, 0))) first_new = t;
        }
        if (crash) {
          ++nsucc;
          if (put(t2, ord_crash) && tail0 == tail - 1) first_new = t2;
        }
        nsucc += (int)uni((uint32_t)selfloop_count_c(L, cu, s));  // Consumer / Terminating stutters
        lvgen += (unsigned)nsucc;
        if (r == 2 || (nsucc == 0 && L.check_deadlock)) {  // an action error or a deadlock: level + 1
          if (inb) evk = min(evk, tree_event_key(level + 1, a.comp0 + (b0 + (u64)(__ffs(inb) - 1)) * 64 + (u64)lane));
        }
        ++head;
        cur = head < tail0 ? nxt : first_new;  // position head was filled by this expansion
        if (head == lvl_end) {  // depth `level` = [lvl_start, lvl_end) is complete and expanded
          if (lane == 0 && nwalk) {
            lvl_d[level] += (unsigned long long)(lvl_end - lvl_start) * nwalk;
            lvl_g[level] += (unsigned long long)lvgen * nwalk;
          }
          lvgen = 0;
          ++level;
          lvl_start = head;
          lvl_end = tail;
          full = full || (tail > head && level >= TREE_MAXLV - 1);
        }
        if (head >= tail || full) break;
      }
#pragma unroll
      for (int m = 0; m < M; ++m) {
        const u64 ci = (b0 + m) * 64 + (u64)lane;
        if (in(m)) a.n_out[ci] = (uint32_t)tail;
      }
      if (full && nwalk) flags |= TREE_OVERFLOW;
      if (nwalk) nexp += (u64)head;  // the walk's code states, expanded once for its components
      maxn = nwalk && (uint32_t)tail > maxn ? (uint32_t)tail : maxn;
      __syncthreads();  // (the next walk clears the table)
    }
  }
  // fold the lanes' flags, the largest component and the least error key, then the per-depth counts
  const unsigned fo = __ballot(flags & TREE_OVERFLOW) ? TREE_OVERFLOW : 0;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) evk = min(evk, (u64)__shfl_xor((unsigned long long)evk, off));
  if (lane == 0) {
    if (fo) atomicOr(a.flags, fo);
    atomicMax(a.max_n, maxn);
    if (evk != ~0ull) atomicMin(a.event, (unsigned long long)evk);
    if (nexp && a.expansions) atomicAdd(&a.expansions[a.nstripe > 1 ? blockIdx.x % (unsigned)a.nstripe : 0], nexp);
  }
  __syncthreads();
  const u64 so = a.nstripe > 1 ? (u64)(blockIdx.x % (unsigned)a.nstripe) * a.stripe : 0;  // this workgroup's copy
  for (int i = lane; i < TREE_MAXLV; i += 64) {
    if (lvl_d[i]) atomicAdd(&a.lvl[so + i], lvl_d[i]);
    if (lvl_g[i]) atomicAdd(&a.lvl_gen[so + i], lvl_g[i]);
  }
}

}  // namespace tlcg
