// pulsar-tlaplus_amd/csrc/tree_body.h -- device body of the component-tree
// engine (tree.h), shared by the precompiled kernels (tree.hip) and the
// run-time specialized ones (jit.cpp): a wavefront runs G components at once,
// one per group of 64 / G lanes, each with its FPSet in LDS.
//   - Producer modelled (CLOSED = false): a component's BFS is a multi-source
//     BFS whose sources are its parent component's states with the
//     component's message appended; states are 32-bit local keys.
//   - Closed (CLOSED = true: no Producer, components too large for a lane of
//     the component engine): a component is the closure of one initial state,
//     states are component codes (component_code.h) and words of type W
//     (u64, or u128 for a > 63-bit layout).
// L is the runtime layout (precompiled kernels) or a constexpr one (jit.cpp),
// in which case every field folds.
#pragma once
#if !defined(__HIPCC_RTC__)
#include "component_code.h"
#include "component_model.h"
#include "kernels.h"
#include "tree.h"
#endif

namespace tlcg {

// CAP states per component, T FPSet slots (a power of 2, load <= CAP / T;
// closed mode scales its table to TLCG_TREE_TSCALE_CLOSED % of CAP instead),
// G components per wavefront.  A component's depth holds ~16 states (P8) or
// fewer, so one component per 64-lane wavefront leaves most lanes idle and
// pays the scalar (exec-mask, loop) instructions once per state; G groups
// share them.
// closed mode: the store holds each state's component code (4 B; the host
// decodes it with the component's messages, tlcg_state_at / copy_states)
// instead of the state word built from it -- G9-deep: the 93-bit words cost
// 21 % of the kernel (TLCG_TREE_NO_STORE, profiles/r03_tree_closed_variants.jsonl).
// 0: words, for A/B
#ifndef TLCG_TREE_CODE_STORE
#define TLCG_TREE_CODE_STORE 1
#endif
// closed mode: a depth of at most half a group's lanes expands in one step
// with one insert (pair mode, in the expansion loop); 0: two inserts, for A/B
#ifndef TLCG_TREE_PAIR
#define TLCG_TREE_PAIR 1
#endif
#ifndef TLCG_TREE_PAIR_OPEN  // (the same in Producer mode; A/B)
#define TLCG_TREE_PAIR_OPEN 0
#endif
// a group of 16 lanes sums its generated successors per depth by a DPP row
// scan (four VALU ops) instead of four ds_bpermute round trips; 0: shuffles, for A/B
#ifndef TLCG_TREE_DPP
#define TLCG_TREE_DPP 1
#endif
// closed mode: each slot displaced by the host's per-bucket table
// (TreeArgs::disp), a perfect hash for the component's code set, so an insert
// takes one CAS instead of a linear-probe chain (G9-deep: 1.00 instead of
// 3.76 probes per insert call, the longest lane of a group); 0: off, for A/B
#ifndef TLCG_TREE_DISP
#define TLCG_TREE_DISP 1
#endif
// closed mode: a state's invariants are evaluated when it is expanded (one
// evaluation per expansion step, the depth's states spread over the group's
// lanes) instead of when it is inserted (one per insert call, two per step
// outside pair mode); every state is expanded once, at the depth after its
// own, so the same states are checked and a violation still reaches the
// least error key (a.event: tree_event_key); 0: at insert, for A/B
// (_OPEN: Producer mode, where a component's entries are expanded too)
#ifndef TLCG_TREE_INV_AT_EXPAND
#define TLCG_TREE_INV_AT_EXPAND 1
#endif
#ifndef TLCG_TREE_INV_AT_EXPAND_OPEN  // (the same in Producer mode)
#define TLCG_TREE_INV_AT_EXPAND_OPEN 1
#endif
#ifndef TLCG_TREE_CAS1  // closed mode: the first CAS outside the probe loop; 0: inside (A/B)
#define TLCG_TREE_CAS1 1
#endif
// (the same in Producer mode, where a collision then goes on to the loop:
// P8 1.857-1.870 -> 1.824-1.826 ms, interleaved on one box,
// profiles/r04_probe_cas1.jsonl; 0 for A/B)
#ifndef TLCG_TREE_CAS1_OPEN
#define TLCG_TREE_CAS1_OPEN 1
#endif
#ifndef TLCG_TREE_MULT  // the slot hash's multiplier (multiply-shift)
#define TLCG_TREE_MULT 0x9E3779B1u
#endif
#ifndef TLCG_TREE_TSCALE_CLOSED
#define TLCG_TREE_TSCALE_CLOSED 100
#endif
// BITS (closed mode, round 6): the FPSet of a component is one bit per slot
// of the host's perfect hash (mult + disp) instead of a code + 1 per slot, with
// a workgroup-shared table own[slot] = the code of the shared code set in that
// slot + 1 (TreeArgs::owner).  FPSet.put(key) is exact for any key: key is
// present iff own[slot(key)] = key + 1 and its bit is set (an LDS atomicOr
// returns the old bit, so two lanes inserting one key agree on which is
// first); a key outside the set raises TREE_OVERFLOW, and the 2048-state pass
// (code + 1 tables, linear probing) takes the model.  A component's table is
// CAP / 8 bytes instead of CAP x 4, so a CU holds more wavefronts.
template <int CAP, int T, int G, bool CLOSED = false, typename W = u64, bool BITS = false>
__device__ __forceinline__ void tree_body(const TreeArgs& a, const Layout& L) {
  static_assert(!BITS || CLOSED, "the bitmap FPSet needs the shared code set (closed mode)");
  constexpr int S = 64 / G;  // lanes per group
  static_assert((T & (T - 1)) == 0 && T >= CAP, "T: a power of 2 >= CAP");
  // FPSet slots per component.  Closed mode: TLCG_TREE_TSCALE_CLOSED % of
  // CAP (a multiple of 16, any size: multiply-shift slot hash), so a CU holds
  // more wavefronts (G9-deep 42.1 -> 35.2 ms at 105 %: 672 slots, 12 instead
  // of 9 workgroups per CU; with the frontier buffer below, 100 % = 640
  // slots measured 31.2 vs 33.6 ms).  Producer mode keeps its power-of-2 T (a smaller
  // table measured slower on P8: 2.34 vs 2.05 ms).  TLCG_TREE_TSCALE (A/B)
  // scales both.
#ifdef TLCG_TREE_TSCALE
  constexpr int TT = (CAP * TLCG_TREE_TSCALE / 100 + 15) / 16 * 16;
#else
  constexpr int TT = CLOSED ? (CAP * TLCG_TREE_TSCALE_CLOSED / 100 + 15) / 16 * 16 : T;
#endif
  static_assert(TT >= CAP, "an FPSet holds a whole component");
  constexpr bool TPOW2 = (TT & (TT - 1)) == 0;
  constexpr int HW = BITS ? (TT + 127) / 128 * 4 : TT;  // words per component's table (BITS: whole uint4s)
  __shared__ uint32_t h[G][HW];      // key + 1, 0 = empty (BITS: one bit per slot)
  __shared__ uint32_t own[BITS ? TT : 1];  // BITS: the code in each slot + 1
#ifndef TLCG_TREE_KEYS_LDS
  // A depth's states are read back from the group's HBM chunk (written
  // before the __syncthreads that ends the insert step, so visible to the
  // workgroup) and re-encoded, so the keys take no LDS and a CU holds more
  // wavefronts: G9-deep 55.7 -> 42.1 ms, P8 2.74 -> 2.08 ms (same box;
  // TLCG_TREE_KEYS_LDS = the keys in LDS, for A/B).
  constexpr int KCAP = 1;
#else
  constexpr int KCAP = CAP;
#endif
  __shared__ uint32_t keys[G][KCAP];  // each component's keys in BFS (depth) order
  // FB: the first FB keys of the depth being expanded and of the next one
  // stay in LDS (two buffers by depth parity), so the expansion reads the
  // store only past them -- no HBM load (behind the previous depth's stores)
  // and no re-encode on the common path.  0 = off.  Closed mode: 16 (G9-deep
  // 35.2 -> 31.2 ms with 640-slot tables, profiles/r02_tree_fb_ab.jsonl; a
  // depth of G9-deep holds 7.5 states on average); Producer mode: 48, in the
  // LDS the 32-bit depth counts for 64 depths leave below the 10 KB that
  // keeps 16 workgroups per CU (P8 1.82-1.85 -> 1.58-1.59 ms; 16 / 24 / 32 /
  // 40 / 48: 1.71 / 1.67 / 1.61-1.62 / 1.59 / 1.58-1.59,
  // profiles/r06_probe_p8_fb.jsonl; in round 2, with 64-bit counts for 128
  // depths, any buffer crossed 10 KB and measured slower)
#ifndef TLCG_TREE_FB
#define TLCG_TREE_FB 16
#endif
#ifndef TLCG_TREE_FB_OPEN
#define TLCG_TREE_FB_OPEN 48
#endif
  // (closed mode's bitmap pass, 16 groups per wavefront: 48 keys; G9-deep
  // 16 / 32 / 48 / 64: 9.0-9.6 / 7.9 / 7.3 / 8.4 ms on one box,
  // profiles/r06_probe_treecb_g.jsonl)
#ifndef TLCG_TREE_FB_BITS
#define TLCG_TREE_FB_BITS 48
#endif
  constexpr int FB = KCAP == CAP ? 0 : CLOSED ? (BITS ? TLCG_TREE_FB_BITS : TLCG_TREE_FB) : TLCG_TREE_FB_OPEN;
  // (a group stride of S (mod 32) words, so that the groups of a half-wave
  // read their buffers on distinct banks, measured slower: G9-deep 7.30-7.35
  // vs 8.01 ms, the padding costs the bitmap pass a workgroup per CU;
  // profiles/r06_probe_tree_fbpad.jsonl)
  constexpr int FBS = FB > 0 ? 2 * FB : 1;
  __shared__ uint32_t fbuf[G * FBS];
  int dbase = 0;  // the first position of the depth being inserted (FB)
  // per-depth counts: 32 bits (a workgroup runs far fewer than 2^32 states
  // at one depth); LDS sums for the first LV depths, global atomics on the
  // workgroup's striped copy past them (Producer mode: deep components are
  // rare and the LDS goes to the frontier buffer)
  typedef unsigned int lvl_t;
#ifndef TLCG_TREE_LVL_DEPTHS_OPEN
#define TLCG_TREE_LVL_DEPTHS_OPEN 64
#endif
  constexpr int LV = CLOSED ? TREE_MAXLV : TLCG_TREE_LVL_DEPTHS_OPEN;
  static_assert(LV <= TREE_MAXLV, "the host sums TREE_MAXLV depths");
  __shared__ lvl_t lvl_d[LV], lvl_g[LV];
  constexpr int ND = CLOSED && TLCG_TREE_DISP ? TREE_DISP : 1;
  __shared__ uint16_t dsp[ND];
  const int lane = threadIdx.x;
  const int g = lane / S, sub = lane % S;
  const u64 gmask = (S == 64 ? ~0ull : ((1ull << S) - 1)) << (g * S);  // my group's lanes
  const u64 below = lanemask_lt() & gmask;
  const int mb = L.msg_sh + L.N * L.mw;  // `messages` (with its length) occupies the low mb bits
  int log2t = 0;
  while ((1 << log2t) < TT) ++log2t;
  for (int i = lane; i < LV; i += 64) lvl_d[i] = lvl_g[i] = 0;
  if constexpr (ND > 1) {
    for (int i = lane; i < ND; i += 64) dsp[i] = a.disp[i];
  }
  if constexpr (BITS) {
    for (int i = lane; i < TT; i += 64) own[i] = a.owner[i];
  }
  __syncthreads();
  unsigned flags = 0;
  uint32_t maxn = 0;
  u64 nexp = 0;  // states this lane's group expanded (its last lane counts them per depth)
  u64 evk = ~0ull;  // this lane's least error key (tree_event_key)
  u64 subtree = 0;  // Producer modelled: the group's component's first message (its subtree), nkv for the root
  // a group's current component and its BFS state (uniform inside the group)
  u64 ci = (u64)blockIdx.x * G + (u64)g;
  const u64 cstep = (u64)gridDim.x * G;
  bool have = false;
  u64 np = 0, pc = 0, e = 0;
  W msgs = 0;
  int j = 0, nprod = 0, n = 0, f0 = 0, d = 0;
  CompMsgs cm{};
  CodeConsts kc{};
  const u64* pst = nullptr;
  const uint8_t* pdep = nullptr;
  u64 pgb = 0, gb = 0;
  W* st = nullptr;
  uint32_t* stc = nullptr;  // (closed mode, TLCG_TREE_CODE_STORE: the chunk as codes)
  u64* par = nullptr;
  uint8_t* dp = nullptr;
  uint32_t* hh = &h[g][0];
  uint32_t* kk = &keys[g][0];
  // insert the group's candidates (pred) at depth dd: LDS CAS on the key, the
  // new ones appended in lane order
  auto insert = [&](bool pred, uint32_t key, u64 pref, int dd) {
    bool isnew = false;
    if (pred) {
      const uint32_t mult = CLOSED ? a.mult : (uint32_t)TLCG_TREE_MULT;
      unsigned s = TPOW2 ? (key * mult) >> (32 - log2t)
                         : (unsigned)(((unsigned long long)(key * mult) * (unsigned)TT) >> 32);
      if constexpr (ND > 1) {
        s += dsp[(key * a.disp_mult) >> 24];
        s = s >= (unsigned)TT ? s - (unsigned)TT : s;
      }
      int p0 = 0;
      // the probe step.  Producer mode: an odd step from a second hash of the
      // key (double hashing; TLCG_TREE_DH=0: 1, linear probing).  A wave's
      // insert waits for its longest probe sequence, and linear probing's
      // primary clusters at the tables' final load (~0.7) made that long:
      // P8 1.62 -> 1.40 ms (profiles/r06_probe_p8_dh.jsonl).  Closed mode
      // places every code at its first slot (the host's perfect hash)
#ifndef TLCG_TREE_DH
#define TLCG_TREE_DH 1
#endif
      const unsigned step = TLCG_TREE_DH && !CLOSED && TPOW2 ? ((key * 0x85EBCA6Bu) >> (32 - log2t)) | 1u : 1u;
      if constexpr (BITS) {
        if (own[s] == key + 1u) {
          const uint32_t bit = 1u << (s & 31);
          isnew = !(atomicOr(&hh[s >> 5], bit) & bit);
        } else {
          flags |= TREE_OVERFLOW;  // not the shared code set: the 2048-state pass takes the model
        }
        p0 = TT;  // (no probe loop)
      } else if constexpr (CLOSED ? TLCG_TREE_CAS1 : TLCG_TREE_CAS1_OPEN) {
        // the first CAS outside the probe loop: with the perfect hash it
        // settles every insert, so the loop is skipped (no lane collides);
        // in Producer mode it settles most
        const uint32_t old = atomicCAS(&hh[s], 0u, key + 1u);
        isnew = old == 0;
        p0 = old == 0 || old == key + 1u ? TT : 1;
        s = TPOW2 ? (s + step) & (TT - 1) : (s + 1 == (unsigned)TT ? 0u : s + 1);
      }
      for (int p = p0; p < TT; ++p) {
        const uint32_t old = atomicCAS(&hh[s], 0u, key + 1u);
        // Producer mode: the probe loop with one exit (P8 2.07 -> 1.99 ms);
        // closed mode: two (G9-deep 31.7 vs 32.5 ms with one;
        // profiles/r02_tree_fb_ab.jsonl)
        if constexpr (!CLOSED) {
          isnew = old == 0;
          if (old == 0 || old == key + 1u) break;
        } else {
          if (old == 0) {
            isnew = true;
            break;
          }
          if (old == key + 1u) break;
        }
        s = TPOW2 ? (s + step) & (TT - 1) : (s + 1 == (unsigned)TT ? 0u : s + 1);
      }
    }
    const u64 m = __ballot(isnew) & gmask;
    const int cnt = __popcll(m);
    // a table of exactly CAP slots is full once the chunk is, and a lane
    // whose probe found neither its key nor an empty slot lost its state: a
    // chunk filled by this insert (or already full) sends the component on --
    // a component of exactly CAP states too, conservatively (the
    // check before the ballot missed the lanes that lost the last free slot
    // to another lane of the same insert); a larger table always has a free
    // slot while the chunk has room
    if constexpr (TT == CAP) {
      if (have && n + cnt >= CAP) flags |= TREE_OVERFLOW;
    }
    if (n + cnt > CAP) {
      if (have) flags |= TREE_OVERFLOW;
    } else if (isnew) {
      const int pos = n + __popcll(m & below);
      if (KCAP == CAP) kk[pos] = key;
      if constexpr (FB > 0) {
        if (pos - dbase < FB) fbuf[g * FBS + (dd & 1) * FB + pos - dbase] = key;
      }
      par[pos] = pref == NO_PARENT ? NO_PARENT : (a.rank_tag | pref);
      if constexpr (CLOSED) {
#ifndef TLCG_TREE_NO_STORE  // (experiment only: what the state words cost)
        if constexpr (TLCG_TREE_CODE_STORE) stc[pos] = key;
        else st[pos] = code_word<W>(L, kc, msgs, key);
#endif
#ifndef TLCG_TREE_NO_INV  // (experiment only: what the invariants cost)
        if (!TLCG_TREE_INV_AT_EXPAND && check_invariants_cb<W>(L, kc, key) >= 0)
          evk = min(evk, tree_event_key(dd, a.comp0 + ci));  // (the host replays the component)
#endif
      } else {
        st[pos] = msgs | ((u64)key << mb);
        dp[pos] = (uint8_t)dd;  // (read by the next layer)
        if (!TLCG_TREE_INV_AT_EXPAND_OPEN && check_invariants_k(L, cm, key) >= 0) evk = min(evk, tree_event_key(dd, subtree));
      }
    }
    n = n + cnt > CAP ? CAP : n + cnt;
  };
  while (true) {
    // a group without a component takes its next one
    if (!have && ci < a.n_comp) {
      for (int i = sub * 4; i < HW; i += S * 4) *reinterpret_cast<uint4*>(&hh[i]) = make_uint4(0, 0, 0, 0);
      if constexpr (CLOSED) {
        np = 1;  // the component's initial state
        const W s0 = init_state<W>(L, a.comp0 + ci);
        msgs = s0 & messages_mask<W>(L);
        cm = comp_msgs_init(L, (u64)s0);  // (`messages` sits in the low word)
        kc = code_consts(L, cm);
#ifdef TLCG_USER_INV
        code_consts_user<W>(L, kc);  // the user invariants' outcome tables of this component
#endif
        if (code_word<W>(L, kc, msgs, code_encode_w<W>(L, s0)) != s0) flags |= TREE_OVERFLOW;  // no code
      } else {
        if (a.layer == 0) {
          np = a.n_init;
          pc = 0;
          j = 0;
        } else {
          const u64 cg = a.comp_base + ci;  // (the layer's component number)
          pc = cg / (u64)L.nkv - a.par_comp_base;
          j = (int)(cg % (u64)L.nkv);
          np = a.par_n[pc];
        }
        pst = a.layer ? a.par_states + pc * CAP : nullptr;
        pdep = a.layer ? a.par_dep + pc * CAP : nullptr;
        pgb = a.par_gbase + pc * CAP;
        const u64 w0 = a.layer == 0 ? init_state(L, 0) : producer_succ(L, pst[0], a.layer - 1, j);
        {  // the subtree: the component's first message (Producer appends, compaction.tla:83-87)
          u64 per = 1;
          for (int l = 1; l < a.layer; ++l) per *= (u64)L.nkv;
          subtree = a.layer == 0 ? (u64)L.nkv : (a.comp_base + ci) / per;
        }
        msgs = (W)(w0 & L.msgs_mask);
        cm = comp_msgs_init(L, w0);        // everything that reads only `messages`
        nprod = cm.len < L.N ? L.nkv : 0;  // Producer's successors (into the children)
        dp = a.dep + ci * CAP;
      }
      st = reinterpret_cast<W*>(a.states) + ci * CAP;
      stc = reinterpret_cast<uint32_t*>(a.states) + ci * CAP;
      par = a.parents + ci * CAP;
      gb = a.gbase + ci * CAP;
      n = f0 = d = 0;
      e = 0;
      have = true;
    }
    if (!__ballot(have)) break;
    __syncthreads();
    // the next depth: the frontier's, or past a gap the next entries'; a
    // component with neither is complete
    if (have && f0 == n) {
      if (e >= np) {  // (the group sits out the rest of this pass)
        if (sub == 0) a.n_out[ci] = (uint32_t)n;
        maxn = n > (int)maxn ? (uint32_t)n : maxn;
        have = false;
        ci += cstep;
      } else {
        d = CLOSED || a.layer == 0 ? 0 : (int)pdep[e] + 1;
      }
    }
    if (have && d >= TREE_MAXLV - 1) flags |= TREE_OVERFLOW;
    // the entries at depth d (parents at depth d - 1; pdep is nondecreasing)
    bool more = have && e < np;
    dbase = f0;  // entries join depth d, which starts at f0
    while (__ballot(more)) {
      const u64 i = e + (u64)sub;
      bool ok = more && i < np;
      uint32_t key = 0;
      u64 pref = NO_PARENT;
      if constexpr (CLOSED) {
        if (ok) key = code_encode_w<W>(L, init_state<W>(L, a.comp0 + ci));
      } else {
        if (ok && a.layer == 0) {
          key = (lkey)(init_state(L, i) >> mb);
        } else if (ok) {
          ok = (int)pdep[i] + 1 == d;
          key = (lkey)(producer_succ(L, pst[i], a.layer - 1, j) >> mb);
          pref = ((pgb + i) << L.ord_bits) | (u64)ordinal_of(L, ACT_PRODUCER, j);
        }
      }
      insert(ok, key, pref, d);
      const int taken = __popcll(__ballot(ok) & gmask);
      e += (u64)taken;
      more = more && taken == S && e < np;
    }
    __syncthreads();
    const int f1 = n;  // depth d = [f0, f1)
    // expand depth d: compactor and BrokerCrash successors at depth d + 1
    unsigned gen = 0;  // (a group's depth generates far fewer than 2^32 successors)
    dbase = f1;  // depth d + 1 starts at f1
    // pair mode (closed, TLCG_TREE_PAIR): a depth of at most S / 2 states
    // runs in one step whose lanes j and j + S/2 both expand state j, the
    // first inserting its compactor successor and the second its BrokerCrash
    // one, so the depth takes one insert instead of two (the idle half of
    // the group does the second); the store order is the same, except when a
    // compactor successor and a BrokerCrash successor of the same depth are one
    // state: then either lane's CAS may take it, so its position and
    // recorded parent may differ from the two-insert order.  Counts, depths and
    // the state set are unaffected, and no trace is read from the tree's
    // parents (an error is reported by the global engine's TLC-order run)
    constexpr bool PAIR = CLOSED ? TLCG_TREE_PAIR : TLCG_TREE_PAIR_OPEN;
    const bool pairm = PAIR && have && f1 - f0 <= S / 2;
    const bool roleb = pairm && sub >= S / 2;  // (pair mode: this lane inserts the BrokerCrash successor)
    for (int b = f0; __ballot(have && b < f1); b += S) {
      const int i = b + (pairm ? (sub & (S / 2 - 1)) : sub);
      const bool ok = have && i < f1;
      uint32_t k = 0;
      if constexpr (FB > 0) {
        if (ok && i - f0 < FB) k = fbuf[g * FBS + (d & 1) * FB + i - f0];
        else if (ok) {
          if constexpr (CLOSED) k = TLCG_TREE_CODE_STORE ? stc[i] : code_encode_w<W>(L, st[i]);
          else k = (uint32_t)((u64)st[i] >> mb);
        }
      } else if constexpr (CLOSED && KCAP != CAP) {
        if (ok) k = TLCG_TREE_CODE_STORE ? stc[i] : code_encode_w<W>(L, st[i]);
      } else if constexpr (KCAP != CAP) {
        if (ok) k = (uint32_t)((u64)st[i] >> mb);
      } else {
        k = ok ? kk[i] : 0;
      }
      uint32_t t = 0, t2 = 0;
      int act = 0, r, nsucc;
      bool crash;
      if constexpr (CLOSED) {
#ifndef TLCG_TREE_NO_INV
        if (TLCG_TREE_INV_AT_EXPAND && ok && check_invariants_cb<W>(L, kc, k) >= 0)
          evk = min(evk, tree_event_key(d, a.comp0 + ci));
#endif
        r = ok ? compactor_step_cb(L, kc, k, &t, &act) : 0;
        crash = ok && crash_step_c(L, k, &t2);
        nsucc = (r == 1) + (int)crash + selfloop_count_c(L, kc, k);
      } else {
        if (TLCG_TREE_INV_AT_EXPAND_OPEN && ok && check_invariants_k(L, cm, k) >= 0) evk = min(evk, tree_event_key(d, subtree));
        r = ok ? compactor_step_k(L, cm, (u64)msgs, k, k_phase(L, k), &t, &act) : 0;
        crash = ok && crash_step_k(L, k, &t2);
        nsucc = nprod + (r == 1) + (int)crash + selfloop_count_k(L, cm, k);
      }
      if (ok && !roleb) {
        gen += (unsigned)nsucc;
        if (r == 2 || (nsucc == 0 && L.check_deadlock)) {
          evk = min(evk, tree_event_key(d + 1, CLOSED ? a.comp0 + ci : subtree));
        }
      }
      const u64 pref = (gb + (u64)i) << L.ord_bits;
      // (one call for the whole wave: the insert ballots across the lanes)
      insert(roleb ? crash : r == 1, roleb ? t2 : t,
             pref | (u64)(roleb ? ordinal_of(L, ACT_CRASH, 0) : ordinal_of(L, act, 0)), d + 1);
      const bool second = crash && !pairm;
      if (!PAIR || __ballot(second)) insert(second, t2, pref | (u64)ordinal_of(L, ACT_CRASH, 0), d + 1);
    }
    // the group's sum of generated successors, added by its last lane
    if constexpr (S == 16 && TLCG_TREE_DPP) {
      // inclusive scan inside the 16-lane row: lane 15 ends with the sum
      gen += (unsigned)__builtin_amdgcn_update_dpp(0, (int)gen, 0x111, 0xf, 0xf, true);  // row_shr:1
      gen += (unsigned)__builtin_amdgcn_update_dpp(0, (int)gen, 0x112, 0xf, 0xf, true);  // row_shr:2
      gen += (unsigned)__builtin_amdgcn_update_dpp(0, (int)gen, 0x114, 0xf, 0xf, true);  // row_shr:4
      gen += (unsigned)__builtin_amdgcn_update_dpp(0, (int)gen, 0x118, 0xf, 0xf, true);  // row_shr:8
    } else {
#pragma unroll
      for (int off = S / 2; off > 0; off >>= 1) gen += __shfl_xor(gen, off);
    }
    if (have && sub == S - 1 && d < TREE_MAXLV && a.count) {
      nexp += (u64)(f1 - f0);
      if (d < LV) {
        atomicAdd(&lvl_d[d], (lvl_t)(f1 - f0));
        atomicAdd(&lvl_g[d], (lvl_t)gen);
      } else {
        const u64 so = a.nstripe > 1 ? (u64)(blockIdx.x % (unsigned)a.nstripe) * a.stripe : 0;
        atomicAdd(&a.lvl[so + d], (unsigned long long)(f1 - f0));
        atomicAdd(&a.lvl_gen[so + d], (unsigned long long)gen);
      }
    }
    __syncthreads();
    if (have) {
      f0 = f1;
      ++d;
    }
    if (__ballot(flags != 0)) break;  // the global engine takes the model
  }
  // fold the lanes' flags and the largest component, then the per-depth counts
  const unsigned fo = __ballot(flags & TREE_OVERFLOW) ? TREE_OVERFLOW : 0;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) maxn = max(maxn, (uint32_t)__shfl_xor(maxn, off));
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) evk = min(evk, (u64)__shfl_xor((unsigned long long)evk, off));
  nexp = wave_sum_u64(nexp);
  if (lane == 0) {
    if (fo) atomicOr(a.flags, fo);
    atomicMax(a.max_n, maxn);
    if (evk != ~0ull) atomicMin(a.event, (unsigned long long)evk);
    if (nexp && a.expansions) atomicAdd(&a.expansions[a.nstripe > 1 ? blockIdx.x % (unsigned)a.nstripe : 0], nexp);
  }
  __syncthreads();
  const u64 so = a.nstripe > 1 ? (u64)(blockIdx.x % (unsigned)a.nstripe) * a.stripe : 0;  // this workgroup's copy
  for (int i = lane; i < LV; i += 64) {
    if (lvl_d[i]) atomicAdd(&a.lvl[so + i], (unsigned long long)lvl_d[i]);
    if (lvl_g[i]) atomicAdd(&a.lvl_gen[so + i], (unsigned long long)lvl_g[i]);
  }
}

}  // namespace tlcg
