// pulsar-tlaplus_amd/csrc/model.h
//
// The compaction spec (/root/reference/compaction.tla) restated over a packed
// 64-bit state word, shared by the gfx950 kernels and the host runtime.
//
// Packed layout (LSB -> MSB; widths are computed from the model constants by
// make_layout(), see DESIGN.md "Data layout"):
//
//   len    bits(N)          Len(messages)                         compaction.tla:57
//   msg[i] N x (kb + vb)    key index | value index << kb; the id is the
//                           position (Init forces msgs[i].id = i, :194;
//                           Producer appends id Len+1, :86)
//   ledger C x (1 + N)      bit0 = "not Nil", bits 1..N = which message
//                           positions the compacted ledger holds.  Ledger
//                           entries are copies of messages[p] kept in
//                           position order (SelectSeq, :119), ids are unique,
//                           so the mask is canonical (<<>> = present, mask 0)
//   p1r    bits(N)          phaseOneResult: 0 = Nil, else readPosition.
//                           latestForKey is a function of messages[1..r]
//                           (:97-98) and messages is append-only, so r alone
//                           determines the record
//   cursor 1+bits(N)+bits(C) present | compactionHorizon | compactedTopicContext
//   phase  3                compactorState (:52-54)
//   hz     bits(N)          compactionHorizon
//   ctx    bits(C)          compactedTopicContext
//   crash  bits(K)          crashTimes
// consumeTimes is never assigned by any action (Consumer is UNCHANGED vars,
// :185-186; every other action keeps it, :87,100,132,139,145,151,165,182,214),
// so it is the constant 0 from Init (:201) and takes no bits.
//
// Every state of the reachable space encodes to exactly one word (canonical),
// so equality of words == equality of TLC states, and the FPSet can store the
// word itself: dedup is exact (no fingerprint collisions).
//
// The word type W is a template parameter: u64 for layouts of <= 63 bits
// (every kernel's fast path), u128 for wider ones (up to 126 bits, e.g.
// CompactionTimesLimit = 12; the wide engine, wide.hip).  Field values
// themselves always fit 64 bits.
#pragma once
#if defined(__HIPCC_RTC__)
// compiled at run time by hipRTC (jit.cpp): the runtime headers are built in
#define TLCG_HD __host__ __device__ __forceinline__
#define TLCG_HDM __host__ __device__ __forceinline__
#else
#include <stdint.h>
#if defined(__HIPCC__) || defined(__HIP__)
#include <hip/hip_runtime.h>
#define TLCG_HD __host__ __device__ __forceinline__
#define TLCG_HDM __host__ __device__ __forceinline__
#else
#define TLCG_HD static inline
#define TLCG_HDM inline
#endif
#endif

namespace tlcg {

typedef uint64_t u64;
typedef unsigned __int128 u128;

// compaction.tla:39-44 (declaration order)
enum Phase { PH_ONE = 0, PH_WRITE, PH_UCTX, PH_UHOR, PH_PERSIST, PH_DELETE };
// Next disjuncts in source order, compaction.tla:216-231
enum Action {
  ACT_PRODUCER = 0, ACT_PHASEONE, ACT_WRITE, ACT_UCTX, ACT_UHOR, ACT_PERSIST,
  ACT_DELETE, ACT_CRASH, ACT_CONSUMER, ACT_TERMINATING, N_ACTIONS
};
// invariants the spec defines (compaction.tla:236,253,259,280)
enum Invariant { INV_TYPESAFE = 0, INV_LEAK = 1, INV_HORIZON = 2, INV_DUPNULL = 3, N_INVARIANT_KINDS };
// three-valued evaluation, as TLC: holds / false / evaluation error
enum Eval { EV_TRUE = 0, EV_FALSE = 1, EV_ERROR = 2 };
// Layout.inv[q] >= INV_USER: the (inv - INV_USER)-th user invariant (user_inv.h)
constexpr int INV_USER = 16;
#ifdef TLCG_USER_INV
// User invariants in the run-time specialized kernels (jit.cpp): user_inv.cpp
// (user_device_source) lowers the compiled program to straight device code,
// defined after these headers; V is a field view of the state (UVWord below,
// UVCode in component_code.h).  Returns EV_TRUE / EV_FALSE / EV_ERROR.
template <class V>
TLCG_HD int tlcg_user_eval(int k, const V& v);
#endif

// TLC's integers are 32-bit: a user invariant's +, -, * or unary - whose
// result leaves -2^31..2^31-1 is an evaluation error ([TLC-ext] the
// Naturals/Integers overflow check, EC.TLC_MODULE_OVERFLOW), not a wrapped
// or 64-bit value (user_inv.h, and the generated device code)
TLCG_HD bool ui_overflows(long long x) { return x < -2147483648LL || x > 2147483647LL; }

struct Layout {
  int32_t N, C, K, ctl;        // MessageSentLimit, CompactionTimesLimit, MaxCrashTimes, ConsumeTimesLimit
  int32_t nk, nv;              // |KeySet|, |ValueSet| incl. NullKey/NullValue at index 0
  int32_t nkv;                 // nk * nv (Producer fan-out)
  int32_t kb, vb, mw;          // bits per key index, value index, message
  int32_t len_sh, len_w;
  int32_t msg_sh;
  int32_t led_sh, led_w;
  int32_t p1r_sh, p1r_w;
  int32_t cur_sh, curh_w, curc_w;
  int32_t ph_sh;
  int32_t hz_sh, hz_w;
  int32_t ctx_sh, ctx_w;
  int32_t cr_sh, cr_w;
  int32_t bits;                // total state bits (<= 63: one u64 word, bit 63 tags FPSet slots;
                               // <= 126: two words, wide.hip)
  int32_t retain, producer, consumer, term_ok, check_deadlock;
  int32_t ord_bits;            // bits of a successor ordinal (Next position)
  int32_t n_inv;
  int32_t inv[8];              // invariant kinds in cfg order (compaction.cfg:25-31); >= INV_USER: user_inv.h
  int32_t defer_inv;           // 1: the cfg has user invariants -- the level's check kernel evaluates
                               // every invariant (check_invariants_all), the expand kernels none
  u64 msgs_mask;               // bits holding `messages` (low word)
  u64 led_present_mask;        // bit0 of every ledger slot (low word)
  u64 msgs_mask_hi;            // the same masks' bits 64..127 (wide layouts)
  u64 led_present_mask_hi;
};

TLCG_HD int bits_for(u64 maxval) {  // bits to represent 0..maxval
  int b = 0;
  while (b < 64 && (maxval >> b) != 0) ++b;
  return b;
}

template <typename W>
TLCG_HD W wmask(int w) {
  return w >= (int)(8 * sizeof(W)) ? ~(W)0 : (((W)1 << w) - 1);
}
template <typename W>
TLCG_HD u64 fget(W s, int sh, int w) {
  return w ? (u64)((s >> sh) & wmask<W>(w)) : 0;
}
template <typename W>
TLCG_HD W fset(W s, int sh, int w, u64 v) {
  if (!w) return s;
  const W m = wmask<W>(w) << sh;
  return (s & ~m) | (((W)v << sh) & m);
}
// a Layout mask (low and high halves) as a W
template <typename W>
TLCG_HD W wide_mask(u64 lo, u64 hi) {
  if constexpr (sizeof(W) == 8) {
    (void)hi;
    return lo;
  } else {
    return (W)lo | ((W)hi << 64);
  }
}
template <typename W>
TLCG_HD W present_mask(const Layout& L) { return wide_mask<W>(L.led_present_mask, L.led_present_mask_hi); }
template <typename W>
TLCG_HD W messages_mask(const Layout& L) { return wide_mask<W>(L.msgs_mask, L.msgs_mask_hi); }

// murmur3 fmix64: a bijection on 64-bit words.  The "fingerprint" of a state
// is mix64(word); since the word is canonical and mix64 invertible, distinct
// states never share a fingerprint.
TLCG_HD u64 mix64(u64 x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}

// ---- field accessors ----
template <typename W> TLCG_HD int st_len(const Layout& L, W s) { return (int)fget(s, L.len_sh, L.len_w); }
template <typename W> TLCG_HD int st_key(const Layout& L, W s, int pos1) { return (int)fget(s, L.msg_sh + (pos1 - 1) * L.mw, L.kb); }
template <typename W> TLCG_HD int st_val(const Layout& L, W s, int pos1) { return (int)fget(s, L.msg_sh + (pos1 - 1) * L.mw + L.kb, L.vb); }
template <typename W> TLCG_HD int st_phase(const Layout& L, W s) { return (int)fget(s, L.ph_sh, 3); }
template <typename W> TLCG_HD int st_p1r(const Layout& L, W s) { return (int)fget(s, L.p1r_sh, L.p1r_w); }
template <typename W> TLCG_HD int st_hz(const Layout& L, W s) { return (int)fget(s, L.hz_sh, L.hz_w); }
template <typename W> TLCG_HD int st_ctx(const Layout& L, W s) { return (int)fget(s, L.ctx_sh, L.ctx_w); }
template <typename W> TLCG_HD int st_crash(const Layout& L, W s) { return (int)fget(s, L.cr_sh, L.cr_w); }
TLCG_HD int led_base(const Layout& L, int j1) { return L.led_sh + (j1 - 1) * L.led_w; }
template <typename W> TLCG_HD int led_present(const Layout& L, W s, int j1) { return (int)((s >> led_base(L, j1)) & 1); }
template <typename W> TLCG_HD u64 led_mask(const Layout& L, W s, int j1) { return fget(s, led_base(L, j1) + 1, L.N); }
template <typename W> TLCG_HD int cur_present(const Layout& L, W s) { return (int)((s >> L.cur_sh) & 1); }
template <typename W> TLCG_HD int cur_h(const Layout& L, W s) { return (int)fget(s, L.cur_sh + 1, L.curh_w); }
template <typename W> TLCG_HD int cur_c(const Layout& L, W s) { return (int)fget(s, L.cur_sh + 1 + L.curh_w, L.curc_w); }

// A field view of a state for the user invariants (user_inv.h: the
// interpreter, and the generated device code): every field a program reads,
// as the accessors above read it from the packed word.  The component
// engines' views (component_code.h UVCode) return the same values from their
// encodings; tlcg_host_user_view_selfcheck compares them on every reachable
// state of whole components.
template <typename W>
struct UVWord {
  const Layout& L;
  W s;
  TLCG_HDM int len() const { return st_len(L, s); }
  TLCG_HDM int key(int i) const { return st_key(L, s, i); }  // key index of messages[i]
  TLCG_HDM int val(int i) const { return st_val(L, s, i); }  // value index
  TLCG_HDM int phase() const { return st_phase(L, s); }
  TLCG_HDM int p1r() const { return st_p1r(L, s); }
  TLCG_HDM int hz() const { return st_hz(L, s); }
  TLCG_HDM int ctx() const { return st_ctx(L, s); }
  TLCG_HDM int crash() const { return st_crash(L, s); }
  TLCG_HDM int curp() const { return cur_present(L, s); }
  TLCG_HDM int curh() const { return cur_h(L, s); }
  TLCG_HDM int curc() const { return cur_c(L, s); }
  TLCG_HDM int ledp(int j) const { return led_present(L, s, j); }
  TLCG_HDM u64 ledm(int j) const { return led_mask(L, s, j); }
};

TLCG_HD int popcount64(u64 x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __popcll(x);
#else
  return __builtin_popcountll(x);
#endif
}
TLCG_HD int highbit64(u64 x) {  // index of the highest set bit, x != 0
#if defined(__HIP_DEVICE_COMPILE__)
  return 63 - __clzll((long long)x);
#else
  return 63 - __builtin_clzll(x);
#endif
}
// user_inv.h U_NTH: the 1-based position of the j-th set bit of m among bits
// 1..63 (bit 64 excluded), 0 when j < 1 or m has fewer set bits
TLCG_HD long long ui_nth(u64 m, long long j) {
  // (the interpreter's; the generated code uses ui_nth_n below.  A scan to
  // the j-th set bit: clearing the lowest bits and a find-first took the
  // specialized kernels from 67 to 90 VGPRs, profiles/r04_probe_uinv5.jsonl)
  const long long want = j;
  long long pos = 0;
  for (int p = 1; p <= 63 && m; ++p, m >>= 1)
    if ((m & 1) && --j == 0) {
      pos = p;
      break;
    }
  return j > 0 || want < 1 ? 0 : pos;
}

// the same for the generated device code, where the layout is a constant: a
// mask within the N message positions (every ledger and Len mask) is scanned
// by N predicated steps, no loop; anything wider falls back to ui_nth.  G9 +
// LatestIsLast 5.42 -> 4.88 ms (the built-in G9: 4.85), + LedgerSorted 24-38
// -> 21.7, all six 47-56 -> 29.9 (profiles/r04_probe_nthn.jsonl)
template <class LL>
TLCG_HD long long ui_nth_n(const LL& L, u64 m, long long j) {
  if (L.N <= 16 && (m >> L.N) == 0) {
    long long pos = 0, cnt = 0;
    for (int p = 1; p <= 16; ++p) {
      if (p > L.N) break;
      const long long b = (long long)((m >> (p - 1)) & 1);
      cnt += b;
      pos = b && cnt == j ? p : pos;
    }
    return j >= 1 ? pos : 0;
  }
  return ui_nth(m, j);
}

template <typename W>
TLCG_HD int highbit(W x) {  // x != 0
  if constexpr (sizeof(W) == 8) {
    return highbit64(x);
  } else {
    const u64 hi = (u64)(x >> 64);
    return hi ? 64 + highbit64(hi) : highbit64((u64)x);
  }
}
template <typename W>
TLCG_HD int popcount(W x) {
  if constexpr (sizeof(W) == 8) return popcount64(x);
  else return popcount64((u64)x) + popcount64((u64)(x >> 64));
}
// slot hash of a state: mix64 (a bijection) of a one-word state; for a wide
// state a mix of both halves (the wide FPSet stores the whole state, so the
// hash only spreads, it never decides equality)
template <typename W>
TLCG_HD u64 mixw(W s) {
  if constexpr (sizeof(W) == 8) return mix64(s);
  else return mix64((u64)s ^ mix64((u64)(s >> 64) + 0x9E3779B97F4A7C15ull));
}

// MaxCompactedLedgerId, compaction.tla:103-106
template <typename W>
TLCG_HD int max_ledger(const Layout& L, W s) {
  const W p = s & present_mask<W>(L);
  if (!p) return 0;
  return (highbit<W>(p) - L.led_sh) / L.led_w + 1;
}

// CompactMessages(messages, phaseOneResult) as a position mask over 1..r,
// compaction.tla:107-119: keep position i iff it is the last occurrence of its
// key in 1..r (i = latestForKey[key], :98 with Max :91), or its key is NullKey
// and RetainNullKey.  Walk r..1 remembering the keys already seen.
template <typename W>
TLCG_HD u64 compact_mask(const Layout& L, W s, int r) {
  u64 seen = 0, mask = 0;
  for (int i = r; i >= 1; --i) {
    int k = st_key(L, s, i);
    if (k == 0) {
      if (L.retain) mask |= 1ull << (i - 1);
    } else if (!((seen >> k) & 1)) {
      seen |= 1ull << k;
      mask |= 1ull << (i - 1);
    }
  }
  return mask;
}

// Initial state number `idx` in TLC's Init enumeration (compaction.tla:188-202):
// messages \in {msgs \in [1..N -> [id, key, value]] : msgs[i].id = i}; message 1
// varies fastest, key faster than value ([TLC-ext] enumeration order).
template <typename W = u64>
TLCG_HD W init_state(const Layout& L, u64 idx) {
  if (L.producer) return 0;  // messages = <<>>, everything else Nil/0/PhaseOne
  W s = fset((W)0, L.len_sh, L.len_w, (u64)L.N);
  for (int i = 1; i <= L.N; ++i) {
    u64 d = idx % (u64)L.nkv;
    idx /= (u64)L.nkv;
    u64 k = d % (u64)L.nk, v = d / (u64)L.nk;
    s = fset(s, L.msg_sh + (i - 1) * L.mw, L.mw, k | (v << L.kb));
  }
  return s;
}

// The inverse of init_state on an initial state: its enumeration number.
template <typename W = u64>
TLCG_HD u64 init_index(const Layout& L, W s) {
  if (L.producer) return 0;
  u64 idx = 0;
  for (int i = L.N; i >= 1; --i)
    idx = idx * (u64)L.nkv + (u64)st_key(L, s, i) + (u64)st_val(L, s, i) * (u64)L.nk;
  return idx;
}

// Successor ordinal = position in TLC's successor enumeration of one state:
// Producer's (key, value) pairs first, then the remaining disjuncts.
TLCG_HD int ordinal_of(const Layout& L, int action, int j) {
  return action == ACT_PRODUCER ? j : L.nkv + action - 1;
}
TLCG_HD int action_of_ordinal(const Layout& L, int ord) {
  return ord < L.nkv ? ACT_PRODUCER : ord - L.nkv + 1;
}

// Producer, compaction.tla:83-87: successor number j (key index j / nv,
// value index j % nv; key outer, value inner).  Caller checks len < N.
template <typename W>
TLCG_HD W producer_succ(const Layout& L, W s, int len, int j) {
  u64 k = (u64)(j / L.nv), v = (u64)(j % L.nv);
  W t = fset(s, L.msg_sh + len * L.mw, L.mw, k | (v << L.kb));
  return fset(t, L.len_sh, L.len_w, (u64)(len + 1));
}

// The six compactor disjuncts (compaction.tla:93-165) are mutually exclusive
// on compactorState, so a state has at most one compactor successor.
// Returns 0 disabled, 1 enabled (*t, *act set), 2 evaluation error (*act set).
template <typename W>
TLCG_HD int compactor_step_ph(const Layout& L, W s, int ph, W* t, int* act) {
  int p1r = st_p1r(L, s);
  switch (ph) {
    case PH_ONE: {  // CompactorPhaseOne, :93-100
      int len = st_len(L, s);
      if (p1r != 0 || len <= 0) return 0;
      W u = fset(s, L.p1r_sh, L.p1r_w, (u64)len);
      *t = fset(u, L.ph_sh, 3, PH_WRITE);
      *act = ACT_PHASEONE;
      return 1;
    }
    case PH_WRITE: {  // CompactorPhaseTwoWrite, :121-132
      if (p1r == 0) return 0;
      int nid = max_ledger(L, s) + 1;
      if (nid > L.C) return 0;  // newCompactedLedgerId \in 1..CompactionTimesLimit
      u64 mask = compact_mask(L, s, p1r);
      W u = fset(s, led_base(L, nid), L.led_w, 1ull | (mask << 1));
      *t = fset(u, L.ph_sh, 3, PH_UCTX);
      *act = ACT_WRITE;
      return 1;
    }
    case PH_UCTX: {  // CompactorPhaseTwoUpdateContext, :135-139
      W u = fset(s, L.ctx_sh, L.ctx_w, (u64)max_ledger(L, s));
      *t = fset(u, L.ph_sh, 3, PH_UHOR);
      *act = ACT_UCTX;
      return 1;
    }
    case PH_UHOR: {  // CompactorPhaseTwoUpdateHorizon, :141-145
      *act = ACT_UHOR;
      if (p1r == 0) return 2;  // phaseOneResult.readPosition of Nil
      W u = fset(s, L.hz_sh, L.hz_w, (u64)p1r);
      *t = fset(u, L.ph_sh, 3, PH_PERSIST);
      return 1;
    }
    case PH_PERSIST: {  // CompactorPhaseTwoPersistCusror, :147-151
      u64 cur = 1ull | ((u64)st_hz(L, s) << 1) | ((u64)st_ctx(L, s) << (1 + L.curh_w));
      W u = fset(s, L.cur_sh, 1 + L.curh_w + L.curc_w, cur);
      *t = fset(u, L.ph_sh, 3, PH_DELETE);
      *act = ACT_PERSIST;
      return 1;
    }
    case PH_DELETE: {  // CompactorPhaseTwoDeleteLedger, :153-165
      *act = ACT_DELETE;
      int m = max_ledger(L, s);
      W u = fset(s, L.ph_sh, 3, PH_ONE);
      u = fset(u, L.p1r_sh, L.p1r_w, 0);
      if (m != 1) {  // oldCompactedLedgerId = m - 1 (Nil when m = 1)
        int old = m - 1;
        if (old < 1) return 2;  // compactedLedgers[old] out of domain
        u = fset(u, led_base(L, old), L.led_w, 0);  // Nil (no-op if already Nil)
      }
      *t = u;
      return 1;
    }
  }
  return 0;
}

template <typename W>
TLCG_HD int compactor_step(const Layout& L, W s, W* t, int* act) {
  return compactor_step_ph(L, s, st_phase(L, s), t, act);
}

// BrokerCrash, compaction.tla:169-182.  Returns 1 if enabled.
template <typename W>
TLCG_HD int crash_step(const Layout& L, W s, W* t) {
  int cr = st_crash(L, s);
  if (cr >= L.K) return 0;
  W u = fset(s, L.cr_sh, L.cr_w, (u64)(cr + 1));
  u = fset(u, L.ph_sh, 3, PH_ONE);
  u = fset(u, L.p1r_sh, L.p1r_w, 0);
  u64 h = 0, c = 0;
  if (cur_present(L, s)) { h = (u64)cur_h(L, s); c = (u64)cur_c(L, s); }
  u = fset(u, L.hz_sh, L.hz_w, h);
  *t = fset(u, L.ctx_sh, L.ctx_w, c);
  return 1;
}

// Terminating, compaction.tla:205-214 (consumeTimes is the constant 0).
template <typename W>
TLCG_HD int terminating_enabled(const Layout& L, W s) {
  return st_len(L, s) == L.N && st_phase(L, s) == PH_WRITE && max_ledger(L, s) == L.C && L.term_ok;
}

// Stuttering successors (Consumer :185-186 when ModelConsumer; Terminating).
// They equal the parent, so they are generated but never new.
template <typename W>
TLCG_HD int selfloop_count(const Layout& L, W s) {
  return (L.consumer ? 1 : 0) + terminating_enabled(L, s);
}

// ---- invariants ----

// TypeSafe, compaction.tla:236-248
template <typename W>
TLCG_HD int inv_typesafe(const Layout& L, W s) {
  int len = st_len(L, s);
  if (len > L.N) return EV_FALSE;
  for (int i = 1; i <= len; ++i)
    if (st_key(L, s, i) >= L.nk || st_val(L, s, i) >= L.nv) return EV_FALSE;
  int r = st_p1r(L, s);
  if (r != 0 && !(r >= 1 && r <= len)) return EV_FALSE;  // latestForKey[k] <= r as well
  if (st_phase(L, s) > PH_DELETE) return EV_FALSE;
  if (st_hz(L, s) > L.N || st_ctx(L, s) > L.C || st_crash(L, s) > L.K) return EV_FALSE;
  if (cur_present(L, s)) {
    int h = cur_h(L, s), c = cur_c(L, s);
    if (!(h >= 1 && h <= L.N && c >= 1 && c <= L.C)) return EV_FALSE;
  }
  return EV_TRUE;
}

// CompactedLedgerLeak, compaction.tla:253
template <typename W>
TLCG_HD int inv_leak(const Layout& L, W s) {
  return popcount<W>(s & present_mask<W>(L)) <= 2 ? EV_TRUE : EV_FALSE;
}

// CompactionHorizonCorrectness, compaction.tla:259-274, read literally.
// Len(messagesBeforeHorizon) (:269) enumerates the function, so messages[i]
// is evaluated for every i <= compactionHorizon before any i is tested: an i
// past Len(messages) is an evaluation error first ([TLC-ext]).
// messagesBeforeHorizon[i] is Nil only for a null key without RetainNullKey
// (:263-266), and then `RetainNullKey => ...` (:271) holds unevaluated; every
// other message, a retained null-key one included, takes the ELSE branch
// (:272-274): some ledger entry with the same key and id >= i (an entry's id
// is its position).  The LET-bound compactedLedgers[compactedTopicContext] is
// evaluated (and can fail) only for an i that reaches it, left to right.
template <typename W>
TLCG_HD int inv_horizon(const Layout& L, W s) {
  int hz = st_hz(L, s), len = st_len(L, s), ctx = st_ctx(L, s);
  if (hz > len) return EV_ERROR;  // messages[len + 1] out of domain
  for (int i = 1; i <= hz; ++i) {
    int k = st_key(L, s, i);
    if (k == 0 && !L.retain) continue;  // messagesBeforeHorizon[i] = Nil
    if (ctx < 1 || ctx > L.C || !led_present(L, s, ctx)) return EV_ERROR;
    u64 m = led_mask(L, s, ctx);
    int found = 0;  // \E j: compactedLedger[j].key = key /\ compactedLedger[j].id >= i
    u64 rest = m >> (i - 1);
    for (int p = i; rest && !found; ++p, rest >>= 1)
      if ((rest & 1) && st_key(L, s, p) == k) found = 1;
    if (!found) return EV_FALSE;
  }
  return EV_TRUE;
}

// DuplicateNullKeyMessage, compaction.tla:280-294: a null-key entry of
// ledger[context] must not equal a message after the horizon.
template <typename W>
TLCG_HD int inv_dupnull(const Layout& L, W s) {
  int ctx = st_ctx(L, s);
  if (!(L.retain && ctx != 0)) return EV_TRUE;
  if (ctx > L.C || !led_present(L, s, ctx)) return EV_ERROR;
  int hz = st_hz(L, s), len = st_len(L, s);
  u64 m = led_mask(L, s, ctx);
  for (int p = 1; p <= L.N; ++p)
    if (((m >> (p - 1)) & 1) && st_key(L, s, p) == 0 && p > hz && p <= len) return EV_FALSE;
  return EV_TRUE;
}

template <typename W>
TLCG_HD int eval_invariant(const Layout& L, int kind, W s) {
  switch (kind) {
    case INV_TYPESAFE: return inv_typesafe(L, s);
    case INV_LEAK: return inv_leak(L, s);
    case INV_HORIZON: return inv_horizon(L, s);
    case INV_DUPNULL: return inv_dupnull(L, s);
  }
  return EV_ERROR;
}

// First failing invariant in cfg order: returns -1 if all hold, else
// (index << 1) | is_error.
template <typename W>
TLCG_HD int check_invariants(const Layout& L, W s) {
  if (L.defer_inv) return -1;  // user invariants: k_user_check (user_inv.h) checks them all, in cfg order
  for (int q = 0; q < L.n_inv; ++q) {
    int r = eval_invariant(L, L.inv[q], s);
    if (r != EV_TRUE) return (q << 1) | (r == EV_ERROR ? 1 : 0);
  }
  return -1;
}

}  // namespace tlcg
