// pulsar-tlaplus_amd/csrc/component_body.h -- device body of the component
// engine (component.h), shared by the precompiled kernel (component.hip) and
// the run-time specialized one (jit.cpp).
#pragma once
#if !defined(__HIPCC_RTC__)
#include "component.h"
#include "component_code.h"
#include "component_model.h"
#include "kernels.h"
#endif

namespace tlcg {

// slot of a local key in a T-slot table (multiply-shift, T need not be a power of 2)
template <int T>
__device__ __forceinline__ unsigned slot_of(uint32_t key, uint32_t mult = 0x9E3779B1u) {
  return (unsigned)(((unsigned long long)(key * mult) * (unsigned)T) >> 32);
}

// bucket of a local key in an NB-bucket table (xorshift-multiply, then
// multiply-shift: the structured local keys spread better than with a bare
// multiply-shift)
template <int NB>
__device__ __forceinline__ unsigned bucket_of(uint32_t k) {
  k ^= k >> 15;
  k *= 0x2c1b3c6du;
  k ^= k >> 12;
  return (unsigned)(((unsigned long long)k * (unsigned)NB) >> 32);
}

// type selection without <type_traits> (hipRTC)
template <bool B, typename A, typename Z> struct tsel { typedef A type; };
template <typename A, typename Z> struct tsel<false, A, Z> { typedef Z type; };

// what a visit of one successor did (component_body)
struct Visit {
  int code;      // -1 seen, -2 does not fit on chip, else slot or bucket (< 2^16) | (first failing invariant + 1) << 16
  uint32_t nw;   // the bucket's new word after an insert
};

// on-chip FPSet slots per component: 1.5 x the capacity (load <= 2/3)
#ifndef TLCG_FPSET_NUM  // on-chip FPSet slots = K * NUM / DEN (tuning hook, jit.cpp)
#define TLCG_FPSET_NUM 3
#define TLCG_FPSET_DEN 2
#endif
template <int K>
struct CompShape { static constexpr int T = (K * TLCG_FPSET_NUM / TLCG_FPSET_DEN + 15) / 16 * 16; };
// FLAT (default): the loop's rare conditions folded so that the scalar unit
// does less exec-mask bookkeeping per expansion -- the per-insert capacity
// check becomes one check per expansion, the action-error, deadlock and
// invariant events one rare branch, and every exit of the BFS loop one exit
// at the end of an expansion.  G9: 7.09 -> 5.79 ms
// (profiles/r02_comp_flat_ab.jsonl).  0: the branching form, for A/B.
#ifndef TLCG_COMP_FLAT
#define TLCG_COMP_FLAT 1
#endif
#if defined(TLCG_BUCKETS) && TLCG_COMP_FLAT  // (the bucket table checks its room per insert)
#undef TLCG_COMP_FLAT
#define TLCG_COMP_FLAT 0
#endif
// component codes: 1.25 x the capacity (load <= 4/5; measured faster than 1.5 x
// at K = 64: 7.20 vs 7.52 ms on G9), and levels tracked on chip up to 32 (a
// deeper component goes on to the cascade), so a 64-lane workgroup takes
// 13.3 KB of LDS: 12 per CU
#ifndef TLCG_CODE_FPSET_NUM
#define TLCG_CODE_FPSET_NUM 5
#define TLCG_CODE_FPSET_DEN 4
#endif
// the queue and the FPSet in lane columns (A/B only: measured slower, G9
// 6.18 vs 5.80 ms, M8 1.251 vs 1.224, with the same SQ_LDS_BANK_CONFLICT
// count -- the conflicts are the 64 lanes' same-address per-level adds, 60
// extra cycles x 20 levels x batches exactly, not the probes: the lanes of
// a wave run isomorphic components in lockstep, so their probes hit one
// slot row; profiles/r03_pmc_component_g9.json)
#ifndef TLCG_LDS_COLS
#define TLCG_LDS_COLS 0
#endif
#ifndef TLCG_CODE_MAXLV
#define TLCG_CODE_MAXLV 32
#endif
// component codes: the store slot of a state holds one 32-bit record
// (comp_record, component.h: the code, the parent's queue position, the
// action) instead of its state word and parent reference (16 B); the host
// rebuilds both from the slot's component (comp_slot_decode).  G9: the two
// 8-B stores cost 1.0 of 5.5 ms (TLCG_NO_STORE, profiles/r03j_probe.jsonl).
// 0: words, for A/B (the host reads TLCG_JIT_DEFINES the same way)
#ifndef TLCG_COMP_CODE_STORE
#define TLCG_COMP_CODE_STORE 1
#endif
#ifndef TLCG_LVL_UNIFORM
#define TLCG_LVL_UNIFORM 0
#endif
// component codes: the invariants of both successors evaluated before their
// FPSet probes, so the VALU work overlaps the probes' LDS round trips (a
// successor found seen evaluated them in vain: 1.34 evaluations per new
// state instead of 1).  Round 3: G9 4.84 -> 4.62 ms, M8 0.575 -> 0.546 ms
// (profiles/r03_comp_spec_inv_ab.jsonl).  Round 4, with the max-ILP
// scheduler (jit.cpp jit_opts) the hiding no longer pays: evaluated on
// insert, G9 4.65-4.69 -> 4.59 ms, G9's 1/8 share 0.645 -> 0.637, M8
// 0.548-0.549 vs 0.550-0.555 (profiles/r04_probe_spec.jsonl); and with user
// invariants, whose VALU work is more than the probes hide, it never paid
// (G9 + LatestIsLast 6.46 -> 5.42 ms, r04_probe_uinv.jsonl).  1: before the
// probes, for A/B
#ifndef TLCG_SPEC_INV
#define TLCG_SPEC_INV 0
#endif
// component codes: the queue entry behind the second successor's first FPSet
// slot read before the first successor's probe (A/B)
#ifndef TLCG_PREFETCH_Q2
#define TLCG_PREFETCH_Q2 0
#endif
template <int K>
struct CodeShape { static constexpr int T = (K * TLCG_CODE_FPSET_NUM / TLCG_CODE_FPSET_DEN + 15) / 16 * 16; };

// the BFS of one wave's components; L is the runtime layout (precompiled
// kernel) or a constexpr one (jit.cpp), in which case every field folds.
// OD: also count TLC's outdegree histogram (a.outdeg; ~9 % of the kernel's
// time on G9, so only when asked for, tlcg_opts.outdegree).
// CODE: the lane's states are component codes (component_code.h, <= 16 bits)
// instead of 32-bit local keys: the queue takes half the LDS, so a CU holds
// more lanes, and the transitions and invariants read fewer fields.
template <int K, bool OD = false, bool CODE = false>
__device__ __forceinline__ void component_body(const CompArgs& a, const Layout& L) {
  constexpr int T = CODE ? CodeShape<K>::T : CompShape<K>::T;
  constexpr int LV = CODE && TLCG_CODE_MAXLV < COMP_MAXLV ? TLCG_CODE_MAXLV : COMP_MAXLV;  // levels tracked
  typedef typename tsel<CODE, uint16_t, uint32_t>::type qword;
  const int lane = threadIdx.x;
#if TLCG_LDS_COLS
  // lane columns: every dword of the queue and of the FPSet belongs to one
  // lane (dword [r][l]), so the sub-dword reads and writes of a wave hit bank
  // l mod 32 whatever slots or positions its lanes touch.  (Rows of 64 bytes
  // put four lanes' slots in one dword: two lanes of a quad at different
  // slots of one bank parity collided, 51 % of the LDS-array cycles of G9
  // were conflicts, profiles/r02_pmc_component.json.)
  constexpr int QPD = 4 / (int)sizeof(qword);     // queue entries per dword
  __shared__ uint32_t qcol[(K + QPD - 1) / QPD][64];
  qword* const ql = reinterpret_cast<qword*>(&qcol[0][lane]);
  // queue entry p of this lane: entry p % QPD of dword [p / QPD][lane]
  auto Q = [&](unsigned p) -> qword& {
    return QPD == 1 ? ql[p << 6] : ql[((p & ~(unsigned)(QPD - 1)) << 6) | (p & (unsigned)(QPD - 1))];
  };
#else
  __shared__ qword q[K][64];                      // FIFO of local keys (word >> msgs_bits) or codes
  auto Q = [&](unsigned p) -> qword& { return q[p][lane]; };
#endif
#ifndef TLCG_BUCKETS  // linear probing over byte slots (the bucketized table measured no faster)
#if TLCG_LDS_COLS
  static_assert(T % 4 == 0, "FPSet slots in whole dwords");
  __shared__ uint32_t hcol[T / 4][64];            // FPSet: slot s of lane l = byte s % 4 of dword [s / 4][l]
  uint8_t(*const h)[64] = reinterpret_cast<uint8_t(*)[64]>(&hcol[0][0]);  // (the whole table, for clearing)
  uint8_t* const hl = reinterpret_cast<uint8_t*>(&hcol[0][lane]);
  auto H = [&](unsigned s) -> uint8_t& { return hl[((s & ~3u) << 6) | (s & 3u)]; };  // 1 + queue position, 0 = empty
#else
  __shared__ uint8_t h[T][64];                    // FPSet: 1 + queue position, 0 = empty
  auto H = [&](unsigned s) -> uint8_t& { return h[s][lane]; };
#endif
#else
  // FPSet: T / 4 buckets of four 1-byte slots (1 + queue position, 0 = empty);
  // bucket b of lane l is the dword hb[b][l], so a wave's bucket reads hit 64
  // distinct banks, and one read shows four candidates, whose queue entries
  // are then read together
  constexpr int NB = T / 4;
  __shared__ uint32_t hb[NB][64];
  uint8_t(*const h)[64] = reinterpret_cast<uint8_t(*)[64]>(&hb[0][0]);  // (the whole table, for clearing)
#endif
  // per level: distinct states (low 32 bits) + successors generated by
  // expanding the level (high 32 bits), one packed 64-bit LDS add per lane and level
  __shared__ unsigned long long lvl_sh[LV];
  const int mb = L.msg_sh + L.N * L.mw;  // `messages` occupies the low mb bits
  if (lane < LV) lvl_sh[lane] = 0;
  u64 gen = 0, dist = 0;
  uint32_t nexp = 0;  // states expanded (of the components that finish here)
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
    CodeConsts ccon{};
    if constexpr (CODE) {
      ccon = code_consts(L, cmsg);
#ifdef TLCG_USER_INV
      code_consts_user(L, ccon);  // the user invariants' outcome tables of this component
#endif
    }
    u64* st = a.store + b * (u64)K * 64 + (u64)lane;
    u64* par = a.parents + b * (u64)K * 64 + (u64)lane;
    const u64 gbase = a.store_base + b * (u64)K * 64 + (u64)lane;
    // wave-uniform bases + 32-bit lane offsets (saddr + voffset stores), and
    // the parent reference of queue position 0 (+ pos << (6 + ord_bits) per position)
    char* const stb = reinterpret_cast<char*>(a.store + b * (u64)K * 64);
    char* const parb = reinterpret_cast<char*>(a.parents + b * (u64)K * 64);
    const u64 pref = a.rank_tag | (gbase << L.ord_bits);
    constexpr bool CREC = CODE && TLCG_COMP_CODE_STORE;  // 32-bit records (comp_record)
    char* const recb = reinterpret_cast<char*>(reinterpret_cast<uint32_t*>(a.store) + b * (u64)K * 64);
    int head = 0, tail = 0, level = 0, lvl_end = 0, lvl_start = 0;
    // alive: the BFS goes on; stop: an error was found, so (like the level
    // loop of the global engine) the lane finishes expanding the current level
    // and stops at its end -- the counts at an error are end-of-level counts
    bool alive = act, ovf = false, stop = false;
    u64 lgen = 0;            // successors generated (the initial state included)
    unsigned lvgen = 0;      // successors generated by expanding the current level
    unsigned ocnt = 0;  // this component's outdegree histogram, 10 bits per bin
    u64 lev = NO_EVENT;
    lkey k0 = act ? (lkey)(s0 >> mb) : 0;
    if constexpr (CODE) {
      const lkey k0c = code_encode(L, k0);
      if (act && code_decode(L, ccon, k0c) != k0) {  // not a code: the 32-bit cascade pass runs it
        ovf = true;
        alive = false;
      }
      k0 = k0c;
    }
    if (act && alive) {
#ifndef TLCG_BUCKETS
      H(slot_of<T>(k0, a.mult)) = 1;
#else
      hb[bucket_of<NB>(k0)][lane] = 1;
#endif
      Q(0) = k0;
      tail = 1;
      if constexpr (CREC) {
        reinterpret_cast<uint32_t*>(recb)[lane] = comp_record(k0, 0, 0);  // (position 0: the root)
      } else {
        st[0] = s0;
        par[0] = NO_PARENT;
      }
      lgen = 1;
      int c;
      if constexpr (CODE) c = check_invariants_direct(L, ccon, k0);
      else c = check_invariants_k(L, cmsg, k0);
      if (c >= 0) {  // an initial state violates: level field 0 sorts before every expansion
        lev = make_comp_event(0, idx0, 0, 0, (c & 1) ? EVK_INV_ERROR : EVK_VIOLATION, c >> 1);
        alive = false;  // level 0 is complete: nothing is expanded
        stop = true;
      }
    }
    lvl_end = tail;
    // the insert of a new state: queue, HBM store + parent log; returns the
    // first failing invariant + 1 (0: all hold)
    auto insert = [&](lkey key, int action, int pos, int pinv = -1) -> int {
      Q(tail) = (qword)key;
#ifndef TLCG_NO_STORE  // (experiment only: measures what the HBM store costs)
      if constexpr (CREC) {
        *reinterpret_cast<uint32_t*>(recb + (unsigned)(tail * 64 + lane) * 4u) = comp_record(key, pos, action);
      } else {
        const unsigned off = (unsigned)(tail * 64 + lane) * 8u;
        lkey lk = key;
        if constexpr (CODE) lk = code_decode(L, ccon, key);
        *reinterpret_cast<u64*>(stb + off) = msgs | ((u64)lk << mb);
        *reinterpret_cast<u64*>(parb + off) = (pref + ((u64)pos << (6 + L.ord_bits))) | (u64)ordinal_of(L, action, 0);
      }
#endif
      ++tail;
#ifdef TLCG_NO_INV  // (experiment only: measures what the invariants cost)
      return 0;
#else
      if (TLCG_SPEC_INV && CODE) return pinv;  // (evaluated before the probe)
      // (FLAT: the user invariants' tables; INV_UNKNOWN is settled in the rare branch)
      if constexpr (CODE && TLCG_COMP_FLAT) return check_invariants_cbt(L, ccon, key) + 1;
      if constexpr (CODE) return check_invariants_cb(L, ccon, key) + 1;
      else return check_invariants_k(L, cmsg, key) + 1;
#endif
    };
#ifndef TLCG_BUCKETS
    // visit one successor whose probe starts at slot `sl` holding `e`: FPSet
    // lookup, insert, invariants (TLC's FPSet.put + check).  (Flags the caller
    // owns are set by the caller: written through the lambda they ended up in
    // scratch memory, read back behind a vmcnt(0) wait on every expansion.)
    auto visit = [&](lkey key, int action, int pos, unsigned sl, unsigned e, int pinv = -1, int qpre = -1) -> Visit {
#ifndef TLCG_PROBE_LOOP_ONLY
      // the first slot outside the loop: most probes end there (an empty
      // slot, or the state itself), so the divergent loop's exec-mask
      // bookkeeping is paid only on a collision
      if (e != 0) {
        if ((qpre >= 0 ? (lkey)qpre : (lkey)Q(e - 1)) == key) return Visit{-1, 0};  // seen
        for (int p = 1; p < T; ++p) {
          sl = sl + 1 == (unsigned)T ? 0 : sl + 1;
          e = H(sl);
          if (e == 0) break;
          if (Q(e - 1) == key) return Visit{-1, 0};  // seen
        }
      }
#else
      for (int p = 0; p < T; ++p) {
        if (e == 0) break;
        if (Q(e - 1) == key) return Visit{-1, 0};  // seen
        sl = sl + 1 == (unsigned)T ? 0 : sl + 1;
        e = H(sl);
      }
#endif
#if !TLCG_COMP_FLAT
      if (tail >= K) return Visit{-2, 0};  // does not fit on chip: cascade
#endif
      H(sl) = (uint8_t)(tail + 1);
      return Visit{(int)sl | (insert(key, action, pos, pinv) << 16), 0};
    };
#else
    // visit one successor whose probe starts at bucket `b` holding `w`: FPSet
    // lookup, insert, invariants (TLC's FPSet.put + check).  The four queue
    // entries a bucket names are read together (unused slots read entry 0 and
    // are masked), a hit among them is a duplicate, else the first empty slot
    // takes the state; a full bucket (rare at load <= 2/3) moves on to the
    // next.  (Flags the caller owns are set by the caller: written through
    // the lambda they ended up in scratch memory, read behind vmcnt(0).)
    auto visit = [&](lkey key, int action, int pos, unsigned b, uint32_t w, int pinv = -1, int = -1) -> Visit {
      for (int step = 0; step < NB; ++step) {
        const unsigned e0 = w & 255u, e1 = (w >> 8) & 255u, e2 = (w >> 16) & 255u, e3 = w >> 24;
        const lkey q0 = Q(e0 ? e0 - 1 : 0), q1 = Q(e1 ? e1 - 1 : 0);
        const lkey q2 = Q(e2 ? e2 - 1 : 0), q3 = Q(e3 ? e3 - 1 : 0);
        if ((e0 && q0 == key) | (e1 && q1 == key) | (e2 && q2 == key) | (e3 && q3 == key)) return Visit{-1, 0};
        const uint32_t z = (w - 0x01010101u) & ~w & 0x80808080u;  // lowest set bit: the first empty slot
        if (z) {
          if (tail >= K) return Visit{-2, 0};  // does not fit on chip: cascade
          const uint32_t nw = w | ((uint32_t)(tail + 1) << (__builtin_ctz(z) & 24));
          hb[b][lane] = nw;
          return Visit{(int)b | (insert(key, action, pos, pinv) << 16), nw};
        }
        b = b + 1 == (unsigned)NB ? 0 : b + 1;
        w = hb[b][lane];
      }
      return Visit{-2, 0};
    };
#endif
    // the caller's side of a visit: overflow, invariant event
    auto settle = [&](Visit vv, int action, int pos) -> int {
      const int v = vv.code;
#if TLCG_COMP_FLAT && !defined(TLCG_BUCKETS)
      if (false) {  // (no -2: the room for two inserts is checked per expansion)
#else
      if (v == -2) {
#endif
        ovf = true;
        alive = false;
        return -1;
      }
      if (!TLCG_COMP_FLAT && v >= 0 && (v >> 16)) {  // (FLAT: the caller's rare branch)
        const int c = (v >> 16) - 1;
        lev = min(lev, make_comp_event(level + 1, idx0, pos, action, (c & 1) ? EVK_INV_ERROR : EVK_VIOLATION, c >> 1));
        stop = true;
      }
      return v < 0 ? -1 : (v & 0xFFFF);
    };
    // the state at the queue head lives in a register; the next one is read
    // from LDS while this one expands
    lkey cur = k0;
#if TLCG_COMP_FLAT
    // FLAT: one exit at the end of an expansion (every break condition
    // folded into it), so the loop pays the exec-mask bookkeeping of one exit
    if (alive) while (true) {
#else
    while (alive && head < tail) {
#endif
      const lkey s = cur;
      const int tail0 = tail;
      // (read unconditionally, clamped into the queue: no masked LDS read)
      const lkey nxt = Q(head + 1 < K ? head + 1 : K - 1);
      int nsucc = 0;
      lkey t = 0;
      int action = 0;
      // compaction.tla:221-226.  Local keys: per-lane dispatch on
      // compactorState (measured no faster: a scalar branch when the wave
      // agrees on the phase; the branch-free compactor_step_k_sel,
      // TLCG_SEL_STEP).  Codes: branch-free (every phase's successor is a few
      // bit operations).  (Measured slower for codes: the FPSet probe as a
      // wave-uniform loop with selects, 8.6 vs 7.1 ms on G9; a slot hash on
      // 24-bit multiplies, 8.7 vs 7.15 ms -- it spreads the codes worse.)
      int ph, r;
      if constexpr (CODE) {
        ph = c_phase(L, s);
        r = compactor_step_cb(L, ccon, s, &t, &action);
      } else {
        ph = k_phase(L, s);
#ifdef TLCG_SEL_STEP
        r = compactor_step_k_sel(L, cmsg, msgs, s, ph, &t, &action);
#else
        r = compactor_step_k(L, cmsg, msgs, s, ph, &t, &action);
#endif
      }
#if !TLCG_COMP_FLAT
      if (r == 2) {  // no successor from the failing action; the others still count (as k_expand)
        lev = min(lev, make_comp_event(level + 1, idx0, head, action, EVK_ACTION_ERROR, action));
        stop = true;
      }
#endif
      lkey t2 = 0;
      bool crash;  // BrokerCrash, compaction.tla:227
      if constexpr (CODE) crash = crash_step_c(L, s, &t2) != 0;
      else crash = crash_step_k(L, s, &t2) != 0;
      // both successors' first FPSet slots (buckets) are read together
#ifndef TLCG_BUCKETS
      const unsigned sl1 = slot_of<T>(t, a.mult), sl2 = slot_of<T>(t2, a.mult);
      const unsigned e1 = H(sl1);  // (unconditional reads; unused when the action is disabled)
      unsigned e2 = H(sl2);
#else
      const unsigned sl1 = bucket_of<NB>(t), sl2 = bucket_of<NB>(t2);
      const uint32_t e1 = r == 1 ? hb[sl1][lane] : 0u;
      uint32_t e2 = crash ? hb[sl2][lane] : 0u;
#endif
#if TLCG_SPEC_INV
      // both successors' invariants evaluated while their first slots are
      // read (most successors are new; the rest evaluate them in vain)
      int pinv1 = -1, pinv2 = -1;
      if constexpr (CODE) {
        pinv1 = check_invariants_cb(L, ccon, t) + 1;
        pinv2 = check_invariants_cb(L, ccon, t2) + 1;
      }
#else
      constexpr int pinv1 = -1, pinv2 = -1;
#endif
#if TLCG_PREFETCH_Q2 && !defined(TLCG_BUCKETS)
      // the queue entry behind the second successor's first slot, read while
      // the first successor probes (valid unless that one takes the slot)
      int q2pre = (int)Q(e2 ? e2 - 1 : 0);
#else
      int q2pre = -1;
#endif
      lkey first_new = 0;
      int ev1 = 0, ev2 = 0;  // FLAT: first failing invariant + 1 of an inserted successor
      if (r == 1) {
        ++nsucc;
        const Visit v1 = visit(t, action, head, sl1, e1, pinv1);
        const int ins = settle(v1, action, head);
        if (ins >= 0) first_new = t;
        ev1 = v1.code >= 0 ? v1.code >> 16 : 0;
#ifndef TLCG_BUCKETS
        if (ins == (int)sl2 && crash) {  // the slot just taken
          e2 = H(sl2);
          q2pre = -1;
        }
#else
        if (ins == (int)sl2) e2 = v1.nw;  // the bucket just written
#endif
      }
      if ((TLCG_COMP_FLAT || alive) && crash) {  // (FLAT: a lane in the loop is alive)
        ++nsucc;
        const Visit v2 = visit(t2, ACT_CRASH, head, sl2, e2, pinv2, q2pre);
        const int ins = settle(v2, ACT_CRASH, head);
        if (ins >= 0 && tail0 == tail - 1) first_new = t2;
        ev2 = v2.code >= 0 ? v2.code >> 16 : 0;
      }
      if constexpr (CODE) nsucc += selfloop_count_c(L, ccon, s);  // Consumer / Terminating stutters
      else nsucc += selfloop_count_k(L, cmsg, s);
      lvgen += (unsigned)nsucc;
      if constexpr (OD) ocnt += 1u << (10 * (tail - tail0));  // new states this expansion discovered (0..2)
#if !TLCG_COMP_FLAT
      (void)ev1;
      (void)ev2;
      if (alive && nsucc == 0 && L.check_deadlock) {
        lev = min(lev, make_comp_event(level + 1, idx0, head, 15, EVK_DEADLOCK, 0));
        stop = true;
      }
#else
      // an action error (no successor from the failing action; the others
      // still count, as k_expand), a deadlock and the successors' invariant
      // events in one rare branch (with an action error and a deadlock, the
      // action error's key, action < 15, is the smaller)
      if ((r == 2) | (nsucc == 0 && L.check_deadlock) | (ev1 != 0) | (ev2 != 0)) {
        if constexpr (CODE) {
          // an outcome table left it to the programs (check_invariants_cbt):
          // one inlined evaluation of both successors here
#pragma nounroll
          for (int i = 0; i < 2; ++i) {
            if ((i ? ev2 : ev1) == INV_UNKNOWN + 1) {
              const int e = check_invariants_direct(L, ccon, i ? t2 : t) + 1;
              if (i) ev2 = e;
              else ev1 = e;
            }
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
#endif
#if TLCG_COMP_FLAT
      ++head;
      cur = head < tail0 ? nxt : first_new;  // position head was filled by this expansion
      bool brk = head >= tail;  // the component ran out
      if (head == lvl_end) {  // level `level` = [lvl_start, lvl_end) is complete, and expanded
#ifndef TLCG_NO_LVL
        {
          const int lvc = level < LV ? level : LV - 1;
          const unsigned long long lv =
              level >= counted ? (unsigned long long)(lvl_end - lvl_start) | ((unsigned long long)lvgen << 32) : 0ull;
#if TLCG_LVL_UNIFORM
          // the lanes of a wave run isomorphic components in lockstep, so all
          // 64 mostly close the same level at once: then one lane adds the
          // wave's sum (a DPP scan per row of 16, the four row sums read
          // into scalars) instead of 64 adds to one LDS address, which the
          // LDS serializes (SQ_LDS_BANK_CONFLICT).  The halves are packed in
          // 16 bits: <= 64 states and <= 256 successors per lane and level (K <= 64)
          const int lv0 = __builtin_amdgcn_readfirstlane(lvc);
          if (K <= 64 && __ballot(lvc == lv0) == ~0ull) {
            unsigned x = level >= counted ? (unsigned)(lvl_end - lvl_start) | (lvgen << 16) : 0u;
            x += (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, true);  // row_shr:1
            x += (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, true);  // row_shr:2
            x += (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, true);  // row_shr:4
            x += (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, true);  // row_shr:8
            const unsigned s = (unsigned)__builtin_amdgcn_readlane((int)x, 15) + (unsigned)__builtin_amdgcn_readlane((int)x, 31) +
                               (unsigned)__builtin_amdgcn_readlane((int)x, 47) + (unsigned)__builtin_amdgcn_readlane((int)x, 63);
            if (lane == 0) atomicAdd(&lvl_sh[lv0], (unsigned long long)(s & 0xFFFFu) | ((unsigned long long)(s >> 16) << 32));
          } else {
            atomicAdd(&lvl_sh[lvc], lv);
          }
#else
          atomicAdd(&lvl_sh[lvc], lv);
#endif
        }
#endif
        lgen += lvgen;
        lvgen = 0;
        ++level;
        lvl_start = head;  // the new level is [head, tail)
        lvl_end = tail;
        const bool deep = level >= LV;  // more levels than tracked on chip: cascade
        ovf = ovf || deep;
        brk = brk || deep || stop;  // stop: an error in the level just expanded, the new level is not expanded
      }
      // room for both successors of the next expansion (checked once per
      // expansion, not per insert: a component of K - 1 or K states goes on
      // to the cascade too)
      const bool full = !brk && tail > K - 2;
      ovf = ovf || full;
      if (brk || full) break;
#else
      if (!alive) break;
      ++head;
      cur = head < tail0 ? nxt : first_new;  // position head was filled by this expansion
      if (head == lvl_end) {  // level `level` = [lvl_start, lvl_end) is complete, and expanded
#ifndef TLCG_NO_LVL  // (experiment only: measures what the per-level counts cost)
        if (level >= counted) atomicAdd(&lvl_sh[level], (unsigned long long)(lvl_end - lvl_start) | ((unsigned long long)lvgen << 32));
#endif
        lgen += lvgen;
        lvgen = 0;
        ++level;
        if (level >= LV) {
          ovf = true;
          break;
        }
        lvl_start = head;  // the new level is [head, tail)
        lvl_end = tail;
        if (stop) break;  // an error in the level just expanded: the new level is not expanded
      }
#endif
    }
    if (act && ovf) {
      // the next pass redoes the component and counts only levels >= `level`
      // (the complete ones were counted here, at their transitions)
      const unsigned long long k = atomicAdd(a.ovf_n, 1ull);
      a.ovf_list[k] = idx0 | ((u64)(level > counted ? level : counted) << 40);
    } else if (act) {
      // the last level [lvl_start, tail) = [head, tail) was discovered, not
      // expanded (empty when the component ran out)
      if (tail > lvl_start && level >= counted) atomicAdd(&lvl_sh[level], (unsigned long long)(tail - lvl_start));
      gen += lgen;
      dist += (u64)tail;
      nexp += (uint32_t)head;
      if constexpr (OD) {
        od0 += ocnt & 1023;
        od1 += (ocnt >> 10) & 1023;
        od2 += ocnt >> 20;
      }
      ev = min(ev, (unsigned long long)lev);
    }
  }
  gen = wave_sum_u64(gen);
  dist = wave_sum_u64(dist);
  const u64 nx = wave_sum_u64(nexp);
  const u64 o0 = wave_sum_u64(od0), o1 = wave_sum_u64(od1), o2 = wave_sum_u64(od2);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) ev = min(ev, (unsigned long long)__shfl_xor(ev, off));
  __syncthreads();
  const u64 so = a.nstripe > 1 ? (u64)(blockIdx.x % (unsigned)a.nstripe) * a.stripe : 0;  // this workgroup's copy
  if (lane == 0) {
    if (nx && a.expansions) atomicAdd(&a.expansions[so], (unsigned long long)nx);
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
