// pulsar-tlaplus_amd/csrc/component_code.h -- the spec's per-state functions
// on *component codes*: a closed component's local keys (component_model.h)
// re-encoded in about half the bits, so a lane's on-chip queue holds 16-bit
// entries and a CU holds more lanes.
//
// Inside a component `messages` is a constant (component_model.h), and then
// four fields of the local key can only ever take two values each:
//   - phaseOneResult.readPosition is Nil or Len(messages): CompactorPhaseOne
//     is its only writer and writes Len(messages) (compaction.tla:96-97);
//     DeleteLedger and BrokerCrash reset it to Nil (:158,:177);
//   - a compacted ledger is Nil or CompactMessages(messages, Len(messages)):
//     CompactorPhaseTwoWrite is its only writer and writes the messages up to
//     phaseOneResult.readPosition = Len(messages) (:124-130); DeleteLedger
//     resets one to Nil (:160-163);
//   - compactionHorizon is 0 or Len(messages): UpdateHorizon copies
//     readPosition (:143), BrokerCrash copies the cursor's horizon or 0
//     (:178-180);
//   - the cursor's horizon is 0 or Len(messages): PersistCursor copies
//     compactionHorizon (:149).
// (SURVEY App.A.1 derives the same facts by hand.)  So a component code keeps
// one bit per two-valued field and the other
// fields as they are (LSB first):
//
//   P   C bits          ledger j present (j = 1..C)
//   R   1               phaseOneResult = Len(messages) (else Nil)
//   H   1               compactionHorizon = Len(messages) (else 0)
//   ph  3               compactorState
//   X   bits(C)         compactedTopicContext
//   CP  1               cursor present
//   CH  1               cursor horizon = Len(messages) (else 0)
//   CC  bits(C)         cursor context
//   CR  bits(K)         crashTimes
//
// The shipped constants (C = 3, K = 1) take 15 bits.  Every transition and
// invariant below is component_model.h's on the decoded key (code_decode):
// tlcg_host_component_selfcheck runs both on every state of whole components
// and checks that each reachable local key encodes and decodes back to itself
// (so the four facts above are checked, not assumed, on every golden cfg).
// The kernel checks the initial state's round trip; a component whose initial
// key does not encode goes to the 32-bit cascade pass.
#pragma once
#if !defined(__HIPCC_RTC__)
#include "component_model.h"
#endif

namespace tlcg {

typedef uint32_t ckey;  // component code

// component_lane.h's per-lane FPSet: LANE_T slots (bits), the slot of code c
// (c < 2^16) under a 24-bit multiplier: bits 24..31 of the low word of
// c x mult (both operands 24-bit: one full-rate v_mul_u32_u24)
constexpr int LANE_T = 256;
TLCG_HD unsigned lane_slot(uint32_t c, uint32_t mult) {
#if defined(__HIP_DEVICE_COMPILE__)
  // (one full-rate v_mul_u32_u24: from the C form the compiler picks the
  // quarter-rate v_mul_lo_u32, __umul24 included)
  uint32_t p;
  asm("v_mul_u32_u24 %0, %1, %2" : "=v"(p) : "v"(c), "v"(mult));
  return p >> 24;
#else
  return ((c & 0xFFFFFFu) * (mult & 0xFFFFFFu)) >> 24;
#endif
}

// field offsets of a code (functions of the layout: constant-fold under hipRTC)
TLCG_HD int cc_r(const Layout& L) { return L.C; }
TLCG_HD int cc_h(const Layout& L) { return L.C + 1; }
TLCG_HD int cc_ph(const Layout& L) { return L.C + 2; }
TLCG_HD int cc_x(const Layout& L) { return L.C + 5; }
TLCG_HD int cc_cp(const Layout& L) { return cc_x(L) + L.ctx_w; }
TLCG_HD int cc_ch(const Layout& L) { return cc_cp(L) + 1; }
TLCG_HD int cc_cc(const Layout& L) { return cc_ch(L) + 1; }
TLCG_HD int cc_cr(const Layout& L) { return cc_cc(L) + L.curc_w; }
TLCG_HD int code_bits(const Layout& L) { return cc_cr(L) + L.cr_w; }

TLCG_HD uint32_t cget(ckey c, int sh, int w) { return (c >> sh) & lmask(w); }
TLCG_HD ckey cset(ckey c, int sh, int w, uint32_t v) {
  const ckey m = lmask(w) << sh;
  return (c & ~m) | ((v << sh) & m);
}

// per-component constants: everything the code functions read besides the code
struct CodeConsts {
  uint32_t len;   // Len(messages)
  lkey ledbits;   // a present ledger's local-key bits at ledger offset 0: 1 | CompactMessages(messages, len) << 1
  int msgs_ok;    // TypeSafe's messages conjunct
  int hz_live;    // CompactionHorizonCorrectness at horizon = len: some position is not skipped
  int hz_false;   // ... and one of them has no witness in CompactMessages(messages, len)
  int dn0, dn1;   // DuplicateNullKeyMessage is FALSE at horizon 0 / len (ledger present)
  u64 msgs;       // the `messages` bits of the word (UVCode)
  u64 utab;       // user invariants' per-component outcome tables (code_consts_user; 0 without)
};

TLCG_HD CodeConsts code_consts(const Layout& L, const CompMsgs& c) {
  CodeConsts k;
  k.msgs = c.msgs;
  k.utab = 0;
  k.len = (uint32_t)c.len;
  const u64 cm = (c.len >= 1 && c.len <= L.N) ? (c.cm >> ((c.len - 1) * L.N)) & nmask(L.N) : 0;
  k.ledbits = (lkey)(1u | (cm << 1));
  k.msgs_ok = c.msgs_ok;
  const int hz = c.len <= L.N ? c.len : L.N;
  const uint32_t live = (uint32_t)nmask(hz) & ~c.skip;
  uint32_t fail = 0;
  for (int i = 0; i < L.N; ++i) fail |= (uint32_t)((cm & ((c.need >> (i * L.N)) & nmask(L.N))) == 0) << i;
  k.hz_live = live != 0;
  k.hz_false = (fail & live) != 0;
  const u64 upto = nmask(c.len < L.N ? c.len : L.N);
  k.dn0 = (cm & c.null_pos & upto) != 0;
  k.dn1 = (cm & c.null_pos & upto & ~nmask(c.len)) != 0;
  return k;
}

// local key -> code (lossy off the reachable space: code_decode checks)
TLCG_HD ckey code_encode(const Layout& L, lkey k) {
  ckey c = 0;
  for (int j = 1; j <= L.C; ++j) c |= (ckey)k_led_present(L, k, j) << (j - 1);
  c |= (ckey)(k_p1r(L, k) != 0) << cc_r(L);
  c |= (ckey)(k_hz(L, k) != 0) << cc_h(L);
  c |= (ckey)k_phase(L, k) << cc_ph(L);
  c |= (ckey)k_ctx(L, k) << cc_x(L);
  c |= (ckey)k_cur_present(L, k) << cc_cp(L);
  c |= (ckey)(k_cur_h(L, k) != 0) << cc_ch(L);
  c |= (ckey)k_cur_c(L, k) << cc_cc(L);
  c |= (ckey)k_crash(L, k) << cc_cr(L);
  return c;
}

// code -> local key
TLCG_HD lkey code_decode(const Layout& L, const CodeConsts& K, ckey c) {
  lkey k = 0;
  for (int j = 1; j <= L.C; ++j)
    if ((c >> (j - 1)) & 1) k |= K.ledbits << k_led_off(L, j);
  if ((c >> cc_r(L)) & 1) k = lset(L, k, L.p1r_sh, L.p1r_w, K.len);
  k = lset(L, k, L.ph_sh, 3, cget(c, cc_ph(L), 3));
  if ((c >> cc_h(L)) & 1) k = lset(L, k, L.hz_sh, L.hz_w, K.len);
  k = lset(L, k, L.ctx_sh, L.ctx_w, cget(c, cc_x(L), L.ctx_w));
  if ((c >> cc_cp(L)) & 1) {
    const lkey h = ((c >> cc_ch(L)) & 1) ? K.len : 0u;
    const lkey cur = 1u | (h << 1) | (cget(c, cc_cc(L), L.curc_w) << (1 + L.curh_w));
    k = lset(L, k, L.cur_sh, 1 + L.curh_w + L.curc_w, cur);
  }
  k = lset(L, k, L.cr_sh, L.cr_w, cget(c, cc_cr(L), L.cr_w));
  return k;
}

// the same for a whole state word of either width (wide layouts, whose
// local keys exceed 32 bits: the component tree's closed mode)
template <typename W>
TLCG_HD ckey code_encode_w(const Layout& L, W s) {
  ckey c = 0;
  for (int j = 1; j <= L.C; ++j) c |= (ckey)led_present<W>(L, s, j) << (j - 1);
  c |= (ckey)(st_p1r<W>(L, s) != 0) << cc_r(L);
  c |= (ckey)(st_hz<W>(L, s) != 0) << cc_h(L);
  c |= (ckey)st_phase<W>(L, s) << cc_ph(L);
  c |= (ckey)st_ctx<W>(L, s) << cc_x(L);
  c |= (ckey)cur_present<W>(L, s) << cc_cp(L);
  c |= (ckey)(cur_h<W>(L, s) != 0) << cc_ch(L);
  c |= (ckey)cur_c<W>(L, s) << cc_cc(L);
  c |= (ckey)st_crash<W>(L, s) << cc_cr(L);
  return c;
}
// code -> the state word msgs | (its local fields); ledbits as in CodeConsts
template <typename W>
TLCG_HD W code_word(const Layout& L, const CodeConsts& K, W msgs, ckey c) {
  W s = msgs;
  for (int j = 1; j <= L.C; ++j)
    if ((c >> (j - 1)) & 1) s = fset<W>(s, led_base(L, j), L.led_w, (u64)K.ledbits);
  if ((c >> cc_r(L)) & 1) s = fset<W>(s, L.p1r_sh, L.p1r_w, K.len);
  s = fset<W>(s, L.ph_sh, 3, cget(c, cc_ph(L), 3));
  if ((c >> cc_h(L)) & 1) s = fset<W>(s, L.hz_sh, L.hz_w, K.len);
  s = fset<W>(s, L.ctx_sh, L.ctx_w, cget(c, cc_x(L), L.ctx_w));
  if ((c >> cc_cp(L)) & 1) {
    const u64 h = ((c >> cc_ch(L)) & 1) ? K.len : 0u;
    s = fset<W>(s, L.cur_sh, 1 + L.curh_w + L.curc_w, 1ull | (h << 1) | ((u64)cget(c, cc_cc(L), L.curc_w) << (1 + L.curh_w)));
  }
  return fset<W>(s, L.cr_sh, L.cr_w, cget(c, cc_cr(L), L.cr_w));
}

// The field view of a code for the user invariants (model.h UVWord): each
// field from the code's bits and the component's constants, as model.h's
// accessors would read it from code_word(msgs, c); a position or ledger index
// outside 1..N / 1..C (which the compiled programs guard against) reads the
// built word itself, so the view agrees with UVWord on every argument.
template <typename W>
struct UVCode {
  const Layout& L;
  const CodeConsts& K;
  ckey c;
  TLCG_HDM W word() const { return code_word<W>(L, K, (W)K.msgs, c); }
  TLCG_HDM int len() const { return (int)K.len; }
  TLCG_HDM int key(int i) const {
    return i >= 1 && i <= L.N ? (int)fget(K.msgs, L.msg_sh + (i - 1) * L.mw, L.kb) : st_key<W>(L, word(), i);
  }
  TLCG_HDM int val(int i) const {
    return i >= 1 && i <= L.N ? (int)fget(K.msgs, L.msg_sh + (i - 1) * L.mw + L.kb, L.vb) : st_val<W>(L, word(), i);
  }
  TLCG_HDM int phase() const { return (int)cget(c, cc_ph(L), 3); }
  TLCG_HDM int p1r() const { return ((c >> cc_r(L)) & 1) ? (int)K.len : 0; }
  TLCG_HDM int hz() const { return ((c >> cc_h(L)) & 1) ? (int)K.len : 0; }
  TLCG_HDM int ctx() const { return (int)cget(c, cc_x(L), L.ctx_w); }
  TLCG_HDM int crash() const { return (int)cget(c, cc_cr(L), L.cr_w); }
  TLCG_HDM int curp() const { return (int)((c >> cc_cp(L)) & 1); }
  TLCG_HDM int curh() const { return ((c >> cc_cp(L)) & 1) && ((c >> cc_ch(L)) & 1) ? (int)K.len : 0; }
  TLCG_HDM int curc() const { return ((c >> cc_cp(L)) & 1) ? (int)cget(c, cc_cc(L), L.curc_w) : 0; }
  TLCG_HDM int ledp(int j) const { return j >= 1 && j <= L.C ? (int)((c >> (j - 1)) & 1) : led_present<W>(L, word(), j); }
  TLCG_HDM u64 ledm(int j) const {
    if (j < 1 || j > L.C) return led_mask<W>(L, word(), j);
    return ((c >> (j - 1)) & 1) ? (u64)(K.ledbits >> 1) : 0ull;
  }
};

// The fields of a state a user invariant's program can read (user_inv.cpp
// user_device_source finds them over the instructions reachable from its
// entry): its code bits, below.  `messages` and Len(messages) are constants
// of a component and take none.
enum UserField : uint32_t {
  UF_PH = 1, UF_R = 2, UF_H = 4, UF_X = 8, UF_CR = 16, UF_CP = 32, UF_CH = 64, UF_CC = 128, UF_LED = 256
};
TLCG_HD uint32_t code_field_mask(const Layout& L, uint32_t f) {
  uint32_t m = 0;
  if (f & UF_LED) m |= lmask(L.C);
  if (f & UF_R) m |= 1u << cc_r(L);
  if (f & UF_H) m |= 1u << cc_h(L);
  if (f & UF_PH) m |= 7u << cc_ph(L);
  if (f & UF_X) m |= lmask(L.ctx_w) << cc_x(L);
  if (f & UF_CP) m |= 1u << cc_cp(L);
  if (f & UF_CH) m |= 1u << cc_ch(L);
  if (f & UF_CC) m |= lmask(L.curc_w) << cc_cc(L);
  if (f & UF_CR) m |= lmask(L.cr_w) << cc_cr(L);
  return m;
}
// the bits of c under mask m, packed (pext); and back (pdep).  Under hipRTC
// m is a constant and the loops fold to a few shifts.
TLCG_HD uint32_t code_pext(ckey c, uint32_t m) {
  uint32_t r = 0;
  int j = 0;
  for (int b = 0; b < 32; ++b)
    if ((m >> b) & 1u) r |= ((c >> b) & 1u) << j++;
  return r;
}
TLCG_HD ckey code_pdep(uint32_t p, uint32_t m) {
  ckey r = 0;
  int j = 0;
  for (int b = 0; b < 32; ++b)
    if ((m >> b) & 1u) r |= ((p >> j++) & 1u) << b;
  return r;
}

// UVCode that notes a read the code alone does not determine: a message
// position outside 1..N or a ledger index outside 1..C reads the word
template <typename W>
struct UVTab : UVCode<W> {
  mutable bool wide = false;
  TLCG_HDM int key(int i) const { wide |= !(i >= 1 && i <= this->L.N); return UVCode<W>::key(i); }
  TLCG_HDM int val(int i) const { wide |= !(i >= 1 && i <= this->L.N); return UVCode<W>::val(i); }
  TLCG_HDM int ledp(int j) const { wide |= !(j >= 1 && j <= this->L.C); return UVCode<W>::ledp(j); }
  TLCG_HDM u64 ledm(int j) const { wide |= !(j >= 1 && j <= this->L.C); return UVCode<W>::ledm(j); }
};

#ifdef TLCG_USER_INV
// Outcome tables of the user invariants (round 5).  Inside a component
// `messages` is a constant, so a user invariant's outcome on a code depends
// only on the code bits of the fields its program reads (tlcg_user_tab_mask)
// and on the component constants it reads.  With at most 4 such bits, the
// outcomes of every pattern of them sit in CodeConsts::utab (2 bits per
// pattern, from bit tlcg_user_tab_off), and each state reads its outcome
// there instead of running the program:
//   - an invariant that reads of the component constants at most Len and the
//     ledger content (CodeConsts len, ledbits) has its tables worked out on
//     the host when the kernels are generated, one per value of the two
//     (tlcg_user_tab_static: a constant array);
//   - one that reads `messages` has its table filled when the component
//     starts, one evaluation per pattern (tlcg_user_tab_dyn).
// An evaluation that read something its pattern and class do not fix
// (UVTab::wide) leaves the value 3, and the states with that pattern run the
// program themselves: the tables are exact on every code.  The four
// tlcg_user_tab_* are generated with the invariants (user_inv.cpp
// user_device_source, which also finds what each program reads).
TLCG_HD int tlcg_user_tab_off(int k);        // bit offset of k's table in utab, or -1 (none)
TLCG_HD uint32_t tlcg_user_tab_mask(int k);  // the code bits k's table is indexed by
TLCG_HD int tlcg_user_tab_dyn(int k);        // 1: k's table is filled per component
TLCG_HD u64 tlcg_user_tab_static(const CodeConsts& K);  // the host-made tables of K's class

template <typename W = u64>
TLCG_HD void code_consts_user(const Layout& L, CodeConsts& K) {
  K.utab = tlcg_user_tab_static(K);
  for (int q = 0; q < L.n_inv; ++q) {
    if (L.inv[q] < INV_USER) continue;
    const int k = L.inv[q] - INV_USER;
    const int off = tlcg_user_tab_off(k);
    if (off < 0 || !tlcg_user_tab_dyn(k)) continue;
    const uint32_t m = tlcg_user_tab_mask(k);
    const int np = 1 << popcount32(m);
    for (int p = 0; p < np; ++p) {
      const UVTab<W> v{{L, K, code_pdep((uint32_t)p, m)}};
      const int r = tlcg_user_eval(k, v);
      K.utab |= (u64)(v.wide ? 3 : r) << (off + 2 * p);
    }
  }
}

// user invariant k on code c: its table, else its program
template <typename W = u64>
TLCG_HD int user_eval_c(const Layout& L, const CodeConsts& K, int k, ckey c) {
  const int off = tlcg_user_tab_off(k);
  if (off >= 0) {
    const int e = (int)((K.utab >> (off + 2 * (int)code_pext(c, tlcg_user_tab_mask(k)))) & 3u);
    if (e != 3) return e;
  }
  return tlcg_user_eval(k, UVCode<W>{L, K, c});
}
#endif

TLCG_HD int c_phase(const Layout& L, ckey c) { return (int)cget(c, cc_ph(L), 3); }
// MaxCompactedLedgerId, compaction.tla:103-106
TLCG_HD int c_max_ledger(const Layout& L, ckey c) {
  const uint32_t p = c & lmask(L.C);
  return p ? highbit32(p) + 1 : 0;
}

// The compactor disjunct, compaction.tla:93-165 (compactor_step_k on codes).
// Returns 0 disabled, 1 enabled (*t, *act set), 2 evaluation error (*act set).
TLCG_HD int compactor_step_c(const Layout& L, const CodeConsts& K, ckey c, int ph, ckey* t, int* act) {
  const uint32_t r = (c >> cc_r(L)) & 1;
  switch (ph) {
    case PH_ONE:  // CompactorPhaseOne, :93-100: readPosition := Len(messages)
      if (r || K.len == 0) return 0;
      *t = cset(c | (1u << cc_r(L)), cc_ph(L), 3, PH_WRITE);
      *act = ACT_PHASEONE;
      return 1;
    case PH_WRITE: {  // CompactorPhaseTwoWrite, :121-132: ledger MaxCompactedLedgerId + 1
      if (!r) return 0;
      const int nid = c_max_ledger(L, c) + 1;
      if (nid > L.C) return 0;
      *t = cset(c | (1u << (nid - 1)), cc_ph(L), 3, PH_UCTX);
      *act = ACT_WRITE;
      return 1;
    }
    case PH_UCTX:  // CompactorPhaseTwoUpdateContext, :135-139
      *t = cset(cset(c, cc_x(L), L.ctx_w, (uint32_t)c_max_ledger(L, c)), cc_ph(L), 3, PH_UHOR);
      *act = ACT_UCTX;
      return 1;
    case PH_UHOR:  // CompactorPhaseTwoUpdateHorizon, :141-145: horizon := readPosition
      *act = ACT_UHOR;
      if (!r) return 2;  // phaseOneResult.readPosition of Nil
      *t = cset(c | (1u << cc_h(L)), cc_ph(L), 3, PH_PERSIST);
      return 1;
    case PH_PERSIST: {  // CompactorPhaseTwoPersistCusror, :147-151: cursor := [horizon, context]
      ckey u = c | (1u << cc_cp(L));
      u = cset(u, cc_ch(L), 1, (c >> cc_h(L)) & 1);
      u = cset(u, cc_cc(L), L.curc_w, cget(c, cc_x(L), L.ctx_w));
      *t = cset(u, cc_ph(L), 3, PH_DELETE);
      *act = ACT_PERSIST;
      return 1;
    }
    case PH_DELETE: {  // CompactorPhaseTwoDeleteLedger, :153-165
      *act = ACT_DELETE;
      const int m = c_max_ledger(L, c);
      ckey u = cset(c & ~(1u << cc_r(L)), cc_ph(L), 3, PH_ONE);
      if (m != 1) {  // oldCompactedLedgerId = m - 1 (Nil when m = 1)
        if (m - 1 < 1) return 2;  // compactedLedgers[old] out of domain
        u &= ~(1u << (m - 2));
      }
      *t = u;
      return 1;
    }
  }
  return 0;
}

// The same disjunct without branches (the kernel's form): every phase's
// successor is a few bit operations on the code, so all six are formed and
// the one of compactorState selected; the phase after ph is ph + 1 (DELETE ->
// ONE).  *act is set when the result is not 0, as compactor_step_c.
TLCG_HD int compactor_step_cb(const Layout& L, const CodeConsts& K, ckey c, ckey* t, int* act) {
  const uint32_t ph = cget(c, cc_ph(L), 3);
  const uint32_t r = (c >> cc_r(L)) & 1, hb = (c >> cc_h(L)) & 1;
  const int m = c_max_ledger(L, c);
  const ckey base = c & ~(7u << cc_ph(L));
  const ckey t_one = base | (1u << cc_r(L));                                   // :96-97
  const ckey t_write = base | (m < L.C ? 1u << m : 0u);                        // :124-130, ledger m + 1
  const ckey t_uctx = cset(base, cc_x(L), L.ctx_w, (uint32_t)m);               // :137
  const ckey t_uhor = base | (1u << cc_h(L));                                  // :143
  const ckey t_pers = cset(cset(base | (1u << cc_cp(L)), cc_ch(L), 1, hb), cc_cc(L), L.curc_w,
                           cget(c, cc_x(L), L.ctx_w));                         // :149
  const ckey t_del = base & ~(1u << cc_r(L)) & ~(m >= 2 ? 1u << (m - 2) : 0u);  // :156-163
  ckey u = t_one;
  int res = (!r && K.len > 0) ? 1 : 0;
  if (ph == PH_WRITE) { u = t_write; res = (r && m < L.C) ? 1 : 0; }
  if (ph == PH_UCTX) { u = t_uctx; res = 1; }
  if (ph == PH_UHOR) { u = t_uhor; res = r ? 1 : 2; }
  if (ph == PH_PERSIST) { u = t_pers; res = 1; }
  if (ph == PH_DELETE) { u = t_del; res = m == 0 ? 2 : 1; }
  if (ph > PH_DELETE) res = 0;
  *t = u | ((ph >= PH_DELETE ? (uint32_t)PH_ONE : ph + 1) << cc_ph(L));
  if (res) *act = ACT_PHASEONE + (int)ph;
  return res;
}

// compactor_step_cb as update masks (round 6, the per-lane kernel
// component_lane.h): the disjunct's successor of code c depends on c only
// through its phase, whether readPosition is set (r) and its largest present
// ledger m (:103-106) -- the bits it sets and clears -- and, for
// PersistCusror, two fields it copies (cursor horizon := horizon, cursor
// context := context, :149).  So each (phase, r, m) has one entry: the bits
// set, the bits cleared, the copied fields' mask and the result (0 disabled,
// 1 enabled, 2 evaluation error), and a lane forms its state's successor as
// (c & ~clear) | set | (copied & mask).  Index ph | r << 3 | m << 4: 64
// entries for C <= 3 (the 16-bit codes of the per-lane kernel).  Checked
// against compactor_step_cb on every code (tlcg_host_component_selfcheck).
constexpr int STEP_TAB = 64;
TLCG_HD u64 compactor_step_entry(const Layout& L, int idx) {
  const int ph = idx & 7, r = (idx >> 3) & 1, m = idx >> 4;
  const uint32_t xm = lmask(L.ctx_w) << cc_x(L), ccm = lmask(L.curc_w) << cc_cc(L);
  uint32_t set = 0, clr = 7u << cc_ph(L), cpy = 0;
  int res = 0;
  if (ph == PH_ONE) {  // :96-97, readPosition := Len (enabled while it is Nil and Len > 0)
    set = 1u << cc_r(L);
    res = r ? 0 : 1;
  } else if (ph == PH_WRITE) {  // :124-130, ledger m + 1
    set = m < L.C ? 1u << m : 0u;
    res = r && m < L.C ? 1 : 0;
  } else if (ph == PH_UCTX) {  // :137, context := m
    clr |= xm;
    set = ((uint32_t)m << cc_x(L)) & xm;
    res = 1;
  } else if (ph == PH_UHOR) {  // :143, horizon := readPosition
    set = 1u << cc_h(L);
    res = r ? 1 : 2;
  } else if (ph == PH_PERSIST) {  // :149, cursor := [horizon, context]
    set = 1u << cc_cp(L);
    clr |= (1u << cc_ch(L)) | ccm;
    cpy = (1u << cc_ch(L)) | ccm;
    res = 1;
  } else if (ph == PH_DELETE) {  // :156-163, readPosition := Nil, ledger m - 1 deleted
    clr |= (1u << cc_r(L)) | (m >= 2 ? 1u << (m - 2) : 0u);
    res = m == 0 ? 2 : 1;
  }
  set |= (ph >= PH_DELETE ? (uint32_t)PH_ONE : (uint32_t)ph + 1) << cc_ph(L);
  return (u64)set | ((u64)clr << 16) | ((u64)cpy << 32) | ((u64)res << 48);
}
// compactor_step_cb through the entries (tab: STEP_TAB of them)
TLCG_HD int compactor_step_tab(const Layout& L, const CodeConsts& K, const u64* tab, ckey c, ckey* t, int* act) {
  const uint32_t ph = cget(c, cc_ph(L), 3), r = (c >> cc_r(L)) & 1;
  const u64 e = tab[ph | (r << 3) | ((uint32_t)c_max_ledger(L, c) << 4)];
  const uint32_t set = (uint32_t)e & 0xFFFFu, clr = (uint32_t)(e >> 16) & 0xFFFFu, cpy = (uint32_t)(e >> 32) & 0xFFFFu;
  const uint32_t copied = (((c >> cc_h(L)) & 1u) << cc_ch(L)) | (cget(c, cc_x(L), L.ctx_w) << cc_cc(L));
  *t = (c & ~clr) | set | (copied & cpy);
  const int res = ph == PH_ONE && K.len == 0 ? 0 : (int)(e >> 48);
  if (res) *act = ACT_PHASEONE + (int)ph;
  return res;
}

// BrokerCrash, compaction.tla:169-182.  Returns 1 if enabled.
TLCG_HD int crash_step_c(const Layout& L, ckey c, ckey* t) {
  const uint32_t cr = cget(c, cc_cr(L), L.cr_w);
  if ((int)cr >= L.K) return 0;
  ckey u = cset(c, cc_cr(L), L.cr_w, cr + 1);
  u = cset(u & ~(1u << cc_r(L)), cc_ph(L), 3, PH_ONE);
  const uint32_t cp = (c >> cc_cp(L)) & 1;
  u = cset(u, cc_h(L), 1, cp ? (c >> cc_ch(L)) & 1 : 0u);
  *t = cset(u, cc_x(L), L.ctx_w, cp ? cget(c, cc_cc(L), L.curc_w) : 0u);
  return 1;
}

// Consumer (:185-186) when modelled, and Terminating (:205-214)
TLCG_HD int selfloop_count_c(const Layout& L, const CodeConsts& K, ckey c) {
  const int term = (int)K.len == L.N && L.term_ok && c_phase(L, c) == PH_WRITE && c_max_ledger(L, c) == L.C;
  return (L.consumer ? 1 : 0) + term;
}

// TypeSafe, compaction.tla:236-248 (inv_typesafe_k on the decoded key)
TLCG_HD int inv_typesafe_c(const Layout& L, const CodeConsts& K, ckey c) {
  const uint32_t r = ((c >> cc_r(L)) & 1) ? K.len : 0u;
  const uint32_t hz = ((c >> cc_h(L)) & 1) ? K.len : 0u;
  const uint32_t h = ((c >> cc_ch(L)) & 1) ? K.len : 0u;
  const int cc = (int)cget(c, cc_cc(L), L.curc_w);
  const bool ok = K.msgs_ok & (r == 0 || r <= K.len) & (c_phase(L, c) <= PH_DELETE) & ((int)hz <= L.N) &
                  ((int)cget(c, cc_x(L), L.ctx_w) <= L.C) & ((int)cget(c, cc_cr(L), L.cr_w) <= L.K) &
                  (!((c >> cc_cp(L)) & 1) || (h >= 1 && (int)h <= L.N && cc >= 1 && cc <= L.C));
  return ok ? EV_TRUE : EV_FALSE;
}

// CompactedLedgerLeak, compaction.tla:253
TLCG_HD int inv_leak_c(const Layout& L, ckey c) { return popcount32(c & lmask(L.C)) <= 2 ? EV_TRUE : EV_FALSE; }

// the ledger compactedTopicContext names exists (else evaluating it fails)
TLCG_HD bool ctx_ledger_ok(const Layout& L, ckey c) {
  const int ctx = (int)cget(c, cc_x(L), L.ctx_w);
  return ctx >= 1 && ctx <= L.C && ((c >> (ctx - 1)) & 1);
}

// CompactionHorizonCorrectness, compaction.tla:259-274 (inv_horizon_k): the
// horizon is 0 (holds) or Len(messages), where the context's ledger, when
// present, holds CompactMessages(messages, Len(messages)) (CodeConsts)
TLCG_HD int inv_horizon_c(const Layout& L, const CodeConsts& K, ckey c) {
  if (!((c >> cc_h(L)) & 1) || K.len == 0) return EV_TRUE;
  if (!K.hz_live) return EV_TRUE;
  if (!ctx_ledger_ok(L, c)) return EV_ERROR;
  return K.hz_false ? EV_FALSE : EV_TRUE;
}

// DuplicateNullKeyMessage, compaction.tla:280-294 (inv_dupnull_k)
TLCG_HD int inv_dupnull_c(const Layout& L, const CodeConsts& K, ckey c) {
  if (!(L.retain && cget(c, cc_x(L), L.ctx_w) != 0)) return EV_TRUE;
  if (!ctx_ledger_ok(L, c)) return EV_ERROR;
  return (((c >> cc_h(L)) & 1) ? K.dn1 : K.dn0) ? EV_FALSE : EV_TRUE;
}

// first failing invariant in cfg order: -1 all hold, else (index << 1) | is_error
template <typename W = u64>
TLCG_HD int check_invariants_c(const Layout& L, const CodeConsts& K, ckey c) {
  for (int q = 0; q < L.n_inv; ++q) {
    int r;
    switch (L.inv[q]) {
      case INV_TYPESAFE: r = inv_typesafe_c(L, K, c); break;
      case INV_LEAK: r = inv_leak_c(L, c); break;
      case INV_HORIZON: r = inv_horizon_c(L, K, c); break;
      case INV_DUPNULL: r = inv_dupnull_c(L, K, c); break;
      default:
        r = EV_ERROR;
#ifdef TLCG_USER_INV
        if (L.inv[q] >= INV_USER) r = user_eval_c<W>(L, K, L.inv[q] - INV_USER, c);
#endif
    }
    if (r != EV_TRUE) return (q << 1) | (r == EV_ERROR ? 1 : 0);
  }
  return -1;
}

// the same without branches (the kernel's form): every invariant's outcome
// formed, then the first failing one in cfg order selected
template <typename W = u64>
TLCG_HD int check_invariants_cb(const Layout& L, const CodeConsts& K, ckey c) {
  const uint32_t hb = (c >> cc_h(L)) & 1;
  const uint32_t X = cget(c, cc_x(L), L.ctx_w);
  const bool ctx_ok = X >= 1 && (int)X <= L.C && ((c >> (X - 1)) & 1);
  const int horizon = (!hb || K.len == 0 || !K.hz_live) ? EV_TRUE : !ctx_ok ? EV_ERROR : K.hz_false ? EV_FALSE : EV_TRUE;
  const int dupnull = !(L.retain && X != 0) ? EV_TRUE : !ctx_ok ? EV_ERROR : (hb ? K.dn1 : K.dn0) ? EV_FALSE : EV_TRUE;
  int res = -1;
  for (int q = L.n_inv - 1; q >= 0; --q) {
    int r = EV_ERROR;
    if (L.inv[q] == INV_TYPESAFE) r = inv_typesafe_c(L, K, c);
    if (L.inv[q] == INV_LEAK) r = inv_leak_c(L, c);
    if (L.inv[q] == INV_HORIZON) r = horizon;
    if (L.inv[q] == INV_DUPNULL) r = dupnull;
#ifdef TLCG_USER_INV
    if (L.inv[q] >= INV_USER) r = user_eval_c<W>(L, K, L.inv[q] - INV_USER, c);
#endif
    if (r != EV_TRUE) res = (q << 1) | (r == EV_ERROR ? 1 : 0);
  }
  return res;
}

// check_invariants_cb for the component kernel's inserts (round 5): the user
// invariants read from their outcome tables only, and a table entry that
// leaves the decision to the program (3, rare) makes the whole answer
// INV_UNKNOWN, which the kernel settles once, in its rare branch, with
// check_invariants_direct.  So the programs are inlined there once instead
// of into every insert (with six user invariants the copies spilled the
// kernel's scalar registers: G9 18.4 ms against 4.9-5.0 with any one of them).
constexpr int INV_UNKNOWN = 0x3FFE;
template <typename W = u64>
TLCG_HD int check_invariants_cbt(const Layout& L, const CodeConsts& K, ckey c) {
#ifdef TLCG_USER_INV
  const uint32_t hb = (c >> cc_h(L)) & 1;
  const uint32_t X = cget(c, cc_x(L), L.ctx_w);
  const bool ctx_ok = X >= 1 && (int)X <= L.C && ((c >> (X - 1)) & 1);
  const int horizon = (!hb || K.len == 0 || !K.hz_live) ? EV_TRUE : !ctx_ok ? EV_ERROR : K.hz_false ? EV_FALSE : EV_TRUE;
  const int dupnull = !(L.retain && X != 0) ? EV_TRUE : !ctx_ok ? EV_ERROR : (hb ? K.dn1 : K.dn0) ? EV_FALSE : EV_TRUE;
  int res = -1;
  bool unknown = false;
  for (int q = L.n_inv - 1; q >= 0; --q) {
    int r = EV_ERROR;
    if (L.inv[q] == INV_TYPESAFE) r = inv_typesafe_c(L, K, c);
    if (L.inv[q] == INV_LEAK) r = inv_leak_c(L, c);
    if (L.inv[q] == INV_HORIZON) r = horizon;
    if (L.inv[q] == INV_DUPNULL) r = dupnull;
    if (L.inv[q] >= INV_USER) {
      const int k = L.inv[q] - INV_USER;
      const int off = tlcg_user_tab_off(k);
      const int e = off >= 0 ? (int)((K.utab >> (off + 2 * (int)code_pext(c, tlcg_user_tab_mask(k)))) & 3u) : 3;
      unknown |= e == 3;
      r = e == 3 ? EV_TRUE : e;
    }
    if (r != EV_TRUE) res = (q << 1) | (r == EV_ERROR ? 1 : 0);
  }
  return unknown ? INV_UNKNOWN : res;
#else
  return check_invariants_cb<W>(L, K, c);
#endif
}

// every invariant in cfg order, the user's by their programs (no tables)
template <typename W = u64>
TLCG_HD int check_invariants_direct(const Layout& L, const CodeConsts& K, ckey c) {
  for (int q = 0; q < L.n_inv; ++q) {
    int r;
    switch (L.inv[q]) {
      case INV_TYPESAFE: r = inv_typesafe_c(L, K, c); break;
      case INV_LEAK: r = inv_leak_c(L, c); break;
      case INV_HORIZON: r = inv_horizon_c(L, K, c); break;
      case INV_DUPNULL: r = inv_dupnull_c(L, K, c); break;
      default:
        r = EV_ERROR;
#ifdef TLCG_USER_INV
        if (L.inv[q] >= INV_USER) r = tlcg_user_eval(L.inv[q] - INV_USER, UVCode<W>{L, K, c});
#endif
    }
    if (r != EV_TRUE) return (q << 1) | (r == EV_ERROR ? 1 : 0);
  }
  return -1;
}

}  // namespace tlcg
