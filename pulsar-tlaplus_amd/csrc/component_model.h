// pulsar-tlaplus_amd/csrc/component_model.h -- the spec's per-state
// functions specialized to one component (component.h), on 32-bit local keys.
//
// Inside a component `messages` is a constant (no enabled action writes it,
// compaction.tla:87,100,132,139,145,151,165,182,186,214).  Two consequences:
//
// 1. A state is its *local key*: the packed word above the `messages` bits
//    (model.h layout: ledgers, phaseOneResult, cursor, phase, horizon,
//    context, crash), k = word >> led_sh.  The component engine admits a
//    model only when that fits 32 bits, so every transition and invariant
//    below runs on 32-bit integers.
// 2. Every sub-expression that reads only `messages` is evaluated once per
//    component (comp_msgs_init) instead of once per state:
//      - Len(messages)                               (:57);
//      - CompactMessages(messages, r) for r = 1..N   (:107-119);
//      - the messages conjunct of TypeSafe           (:238);
//      - for CompactionHorizonCorrectness (:259-274), per position i, which
//        ledger positions witness it: key(p) = key(i) /\ p >= i (an entry's
//        id is its position; the ELSE branch, :272-274, a retained null key
//        included), and which positions are skipped (null key, not retained);
//      - the null-key positions DuplicateNullKeyMessage (:280-294) reads.
//
// The results are exactly model.h's on the word msgs | k << led_sh (same
// successor, same three-valued invariant outcome in cfg order):
// tlcg_host_component_selfcheck compares the two on whole components.
#pragma once
#if !defined(__HIPCC_RTC__)
#include "model.h"
#endif

namespace tlcg {

typedef uint32_t lkey;  // local key

struct CompMsgs {
  u64 cm;             // CompactMessages for r = 1..N: N bits at (r - 1) * N
  u64 need;           // horizon witnesses of position i = 1..N: N bits at (i - 1) * N (a position p >= i with key(p) = key(i))
  uint32_t skip;      // positions whose messagesBeforeHorizon entry is Nil (null key, not retained)
  uint32_t null_pos;  // positions 1..Len holding NullKey
  u64 hwit;           // N <= 4: for each ledger position mask m, the positions it witnesses: N bits at m * N
  int len;            // Len(messages)
  int msgs_ok;        // TypeSafe's messages conjunct (and Len(messages) <= N)
  u64 msgs;           // the `messages` bits of the word (user invariants: model.h UVWord)
};

TLCG_HD u64 nmask(int n) { return n >= 64 ? ~0ull : ((1ull << n) - 1); }
TLCG_HD uint32_t lmask(int w) { return w >= 32 ? ~0u : ((1u << w) - 1); }

TLCG_HD CompMsgs comp_msgs_init(const Layout& L, u64 s) {
  CompMsgs c;
  c.msgs = s & L.msgs_mask;
  c.len = st_len(L, s);
  c.cm = c.need = 0;
  c.skip = c.null_pos = 0;
  c.msgs_ok = c.len <= L.N;
  // positions 1..N on the raw bits, exactly as model.h reads them
  for (int i = 1; i <= L.N; ++i) {
    const int k = st_key(L, s, i);
    if (i <= c.len && (k >= L.nk || st_val(L, s, i) >= L.nv)) c.msgs_ok = 0;
    c.cm |= compact_mask(L, s, i) << ((i - 1) * L.N);
    if (k == 0 && i <= c.len) c.null_pos |= 1u << (i - 1);
    if (k == 0 && !L.retain) {
      c.skip |= 1u << (i - 1);  // messagesBeforeHorizon[i] = Nil
    } else {
      // the ELSE branch (:272-274), a retained null key included: ledger
      // positions p >= i holding the same key
      u64 w = 0;
      for (int p = i; p <= L.N; ++p)
        if (st_key(L, s, p) == k) w |= 1ull << (p - 1);
      c.need |= w << ((i - 1) * L.N);
    }
  }
  // the witness table: CompactionHorizonCorrectness on a ledger mask m is one
  // lookup (N x 2^N bits <= 64)
  c.hwit = 0;
  if (L.N <= 4)
    for (u64 m = 0; m < (1ull << L.N); ++m)
      for (int i = 0; i < L.N; ++i)
        if (m & ((c.need >> (i * L.N)) & nmask(L.N))) c.hwit |= 1ull << (m * L.N + i);
  return c;
}

// ---- fields of a local key (model.h accessors shifted down by led_sh) ----
TLCG_HD lkey lget(const Layout& L, lkey k, int sh, int w) { return w ? (k >> (sh - L.led_sh)) & lmask(w) : 0; }
TLCG_HD lkey lset(const Layout& L, lkey k, int sh, int w, lkey v) {
  if (!w) return k;
  const lkey m = lmask(w) << (sh - L.led_sh);
  return (k & ~m) | ((v << (sh - L.led_sh)) & m);
}
TLCG_HD int k_phase(const Layout& L, lkey k) { return (int)lget(L, k, L.ph_sh, 3); }
TLCG_HD int k_p1r(const Layout& L, lkey k) { return (int)lget(L, k, L.p1r_sh, L.p1r_w); }
TLCG_HD int k_hz(const Layout& L, lkey k) { return (int)lget(L, k, L.hz_sh, L.hz_w); }
TLCG_HD int k_ctx(const Layout& L, lkey k) { return (int)lget(L, k, L.ctx_sh, L.ctx_w); }
TLCG_HD int k_crash(const Layout& L, lkey k) { return (int)lget(L, k, L.cr_sh, L.cr_w); }
TLCG_HD int k_led_off(const Layout& L, int j1) { return (j1 - 1) * L.led_w; }  // ledger j1, local bit offset
TLCG_HD int k_led_present(const Layout& L, lkey k, int j1) { return (int)((k >> k_led_off(L, j1)) & 1); }
TLCG_HD lkey k_led_mask(const Layout& L, lkey k, int j1) { return (k >> (k_led_off(L, j1) + 1)) & lmask(L.N); }
TLCG_HD lkey k_present_mask(const Layout& L) { return (lkey)(L.led_present_mask >> L.led_sh); }
TLCG_HD int k_cur_present(const Layout& L, lkey k) { return (int)((k >> (L.cur_sh - L.led_sh)) & 1); }
TLCG_HD int k_cur_h(const Layout& L, lkey k) { return (int)lget(L, k, L.cur_sh + 1, L.curh_w); }
TLCG_HD int k_cur_c(const Layout& L, lkey k) { return (int)lget(L, k, L.cur_sh + 1 + L.curh_w, L.curc_w); }
TLCG_HD int highbit32(uint32_t x) {  // x != 0
#if defined(__HIP_DEVICE_COMPILE__)
  return 31 - __clz((int)x);
#else
  return 31 - __builtin_clz(x);
#endif
}
TLCG_HD int popcount32(uint32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __popc(x);
#else
  return __builtin_popcount(x);
#endif
}
// MaxCompactedLedgerId, compaction.tla:103-106
TLCG_HD int k_max_ledger(const Layout& L, lkey k) {
  const lkey p = k & k_present_mask(L);
  return p ? highbit32(p) / L.led_w + 1 : 0;
}

// ---- Next disjuncts on local keys (model.h compactor_step_ph / crash_step) ----

// The compactor disjunct, compaction.tla:93-165.  `msgs` rebuilds the whole
// word for the one case that needs more than the precomputed facts.
// Returns 0 disabled, 1 enabled (*t, *act set), 2 evaluation error (*act set).
TLCG_HD int compactor_step_k(const Layout& L, const CompMsgs& c, u64 msgs, lkey k, int ph, lkey* t, int* act) {
  const int p1r = k_p1r(L, k);
  switch (ph) {
    case PH_ONE: {  // CompactorPhaseOne, :93-100
      if (p1r != 0 || c.len <= 0) return 0;
      *t = lset(L, lset(L, k, L.p1r_sh, L.p1r_w, (lkey)c.len), L.ph_sh, 3, PH_WRITE);
      *act = ACT_PHASEONE;
      return 1;
    }
    case PH_WRITE: {  // CompactorPhaseTwoWrite, :121-132
      if (p1r == 0) return 0;
      const int nid = k_max_ledger(L, k) + 1;
      if (nid > L.C) return 0;
      const u64 mask = p1r <= L.N ? (c.cm >> ((p1r - 1) * L.N)) & nmask(L.N)
                                  : compact_mask(L, msgs | ((u64)k << L.led_sh), p1r);
      const lkey u = lset(L, k, led_base(L, nid), L.led_w, (lkey)(1ull | (mask << 1)));
      *t = lset(L, u, L.ph_sh, 3, PH_UCTX);
      *act = ACT_WRITE;
      return 1;
    }
    case PH_UCTX: {  // CompactorPhaseTwoUpdateContext, :135-139
      *t = lset(L, lset(L, k, L.ctx_sh, L.ctx_w, (lkey)k_max_ledger(L, k)), L.ph_sh, 3, PH_UHOR);
      *act = ACT_UCTX;
      return 1;
    }
    case PH_UHOR: {  // CompactorPhaseTwoUpdateHorizon, :141-145
      *act = ACT_UHOR;
      if (p1r == 0) return 2;  // phaseOneResult.readPosition of Nil
      *t = lset(L, lset(L, k, L.hz_sh, L.hz_w, (lkey)p1r), L.ph_sh, 3, PH_PERSIST);
      return 1;
    }
    case PH_PERSIST: {  // CompactorPhaseTwoPersistCusror, :147-151
      const lkey cur = 1u | ((lkey)k_hz(L, k) << 1) | ((lkey)k_ctx(L, k) << (1 + L.curh_w));
      *t = lset(L, lset(L, k, L.cur_sh, 1 + L.curh_w + L.curc_w, cur), L.ph_sh, 3, PH_DELETE);
      *act = ACT_PERSIST;
      return 1;
    }
    case PH_DELETE: {  // CompactorPhaseTwoDeleteLedger, :153-165
      *act = ACT_DELETE;
      const int m = k_max_ledger(L, k);
      lkey u = lset(L, lset(L, k, L.ph_sh, 3, PH_ONE), L.p1r_sh, L.p1r_w, 0);
      if (m != 1) {  // oldCompactedLedgerId = m - 1 (Nil when m = 1)
        if (m - 1 < 1) return 2;  // compactedLedgers[old] out of domain
        u = lset(L, u, led_base(L, m - 1), L.led_w, 0);
      }
      *t = u;
      return 1;
    }
  }
  return 0;
}

// The same disjunct without branches on compactorState: every phase's
// successor is formed and the one of `ph` selected, so the lanes of a wave
// never diverge here (same results as compactor_step_k; the selfcheck and the
// golden tests run whichever the kernel uses).
TLCG_HD int compactor_step_k_sel(const Layout& L, const CompMsgs& c, u64 msgs, lkey k, int ph, lkey* t, int* act) {
  const int p1r = k_p1r(L, k);
  const int m = k_max_ledger(L, k);
  const lkey to_ph = ~(lmask(3) << (L.ph_sh - L.led_sh));
  const lkey base = k & to_ph;
  auto with_ph = [&](lkey x, int p) { return (x & to_ph) | ((lkey)p << (L.ph_sh - L.led_sh)); };
  // PhaseOne (:93-100)
  const lkey t_one = with_ph(lset(L, base, L.p1r_sh, L.p1r_w, (lkey)c.len), PH_WRITE);
  const bool en_one = p1r == 0 && c.len > 0;
  // PhaseTwoWrite (:121-132); p1r <= N: the precomputed CompactMessages
  const int nid = m + 1;
  const int r1 = p1r > 0 ? p1r - 1 : 0;
  u64 mask = (c.cm >> (r1 * L.N)) & nmask(L.N);
  if (p1r > L.N) mask = compact_mask(L, msgs | ((u64)k << L.led_sh), p1r);
  const int nid_c = nid <= L.C ? nid : L.C;  // (a disabled Write forms a dummy ledger)
  const lkey t_write = with_ph(lset(L, base, led_base(L, nid_c), L.led_w, (lkey)(1ull | (mask << 1))), PH_UCTX);
  const bool en_write = p1r != 0 && nid <= L.C;
  // UpdateContext (:135-139), UpdateHorizon (:141-145)
  const lkey t_uctx = with_ph(lset(L, base, L.ctx_sh, L.ctx_w, (lkey)m), PH_UHOR);
  const lkey t_uhor = with_ph(lset(L, base, L.hz_sh, L.hz_w, (lkey)p1r), PH_PERSIST);
  // PersistCusror (:147-151)
  const lkey cur = 1u | ((lkey)k_hz(L, k) << 1) | ((lkey)k_ctx(L, k) << (1 + L.curh_w));
  const lkey t_pers = with_ph(lset(L, base, L.cur_sh, 1 + L.curh_w + L.curc_w, cur), PH_DELETE);
  // DeleteLedger (:153-165): ledger m - 1 cleared unless m = 1
  const lkey d0 = with_ph(lset(L, base, L.p1r_sh, L.p1r_w, 0), PH_ONE);
  const int old = m - 1 >= 1 ? m - 1 : 1;
  const lkey t_del = m != 1 ? lset(L, d0, led_base(L, old), L.led_w, 0) : d0;
  lkey r = t_one;
  int a = ACT_PHASEONE, res = en_one ? 1 : 0;
  if (ph == PH_WRITE) { r = t_write; a = ACT_WRITE; res = en_write ? 1 : 0; }
  if (ph == PH_UCTX) { r = t_uctx; a = ACT_UCTX; res = 1; }
  if (ph == PH_UHOR) { r = t_uhor; a = ACT_UHOR; res = p1r == 0 ? 2 : 1; }
  if (ph == PH_PERSIST) { r = t_pers; a = ACT_PERSIST; res = 1; }
  if (ph == PH_DELETE) { r = t_del; a = ACT_DELETE; res = m != 1 && m - 1 < 1 ? 2 : 1; }
  if (ph > PH_DELETE) res = 0;
  *t = r;
  if (res) *act = a;
  return res;
}

// BrokerCrash, compaction.tla:169-182.  Returns 1 if enabled.
TLCG_HD int crash_step_k(const Layout& L, lkey k, lkey* t) {
  const int cr = k_crash(L, k);
  if (cr >= L.K) return 0;
  lkey u = lset(L, k, L.cr_sh, L.cr_w, (lkey)(cr + 1));
  u = lset(L, u, L.ph_sh, 3, PH_ONE);
  u = lset(L, u, L.p1r_sh, L.p1r_w, 0);
  lkey h = 0, cc = 0;
  if (k_cur_present(L, k)) {
    h = (lkey)k_cur_h(L, k);
    cc = (lkey)k_cur_c(L, k);
  }
  u = lset(L, u, L.hz_sh, L.hz_w, h);
  *t = lset(L, u, L.ctx_sh, L.ctx_w, cc);
  return 1;
}

// Consumer (:185-186) when modelled, and Terminating (:205-214)
TLCG_HD int selfloop_count_k(const Layout& L, const CompMsgs& c, lkey k) {
  const int term = c.len == L.N && L.term_ok && k_phase(L, k) == PH_WRITE && k_max_ledger(L, k) == L.C;
  return (L.consumer ? 1 : 0) + term;
}

// ---- invariants on local keys ----

// TypeSafe, compaction.tla:236-248 (model.h inv_typesafe); one conjunction,
// no early exits (TypeSafe has no evaluation-error cases)
TLCG_HD int inv_typesafe_k(const Layout& L, const CompMsgs& c, lkey k) {
  const int r = k_p1r(L, k), h = k_cur_h(L, k), cc = k_cur_c(L, k);
  const bool ok = c.msgs_ok & (r == 0 || r <= c.len) & (k_phase(L, k) <= PH_DELETE) & (k_hz(L, k) <= L.N) &
                  (k_ctx(L, k) <= L.C) & (k_crash(L, k) <= L.K) &
                  (!k_cur_present(L, k) || (h >= 1 && h <= L.N && cc >= 1 && cc <= L.C));
  return ok ? EV_TRUE : EV_FALSE;
}

// CompactedLedgerLeak, compaction.tla:253
TLCG_HD int inv_leak_k(const Layout& L, lkey k) {
  return popcount32(k & k_present_mask(L)) <= 2 ? EV_TRUE : EV_FALSE;
}

// CompactionHorizonCorrectness, compaction.tla:259-274 (model.h inv_horizon):
// positions i = 1..hz in order; the first one that decides wins.
TLCG_HD int inv_horizon_k(const Layout& L, const CompMsgs& c, lkey k) {
  const int hz = k_hz(L, k);
  if (hz == 0) return EV_TRUE;
  if (hz > c.len) return EV_ERROR;  // Len(messagesBeforeHorizon) evaluates messages[len + 1]
  const uint32_t live = (uint32_t)nmask(hz) & ~c.skip;
  if (live) {
    const int ctx = k_ctx(L, k);
    // the first live position evaluates compactedLedgers[ctx]
    if (ctx < 1 || ctx > L.C || !k_led_present(L, k, ctx)) return EV_ERROR;
    const u64 m = k_led_mask(L, k, ctx);
    uint32_t fail = 0;  // live positions without a witness in the ledger
#ifndef TLCG_HWIT_OFF  // (A/B hook: the loop instead of the table)
    if (L.N <= 4) {
      fail = ~(uint32_t)(c.hwit >> (m * L.N)) & (uint32_t)nmask(L.N);
    } else
#endif
    {
      for (int i = 0; i < L.N; ++i) fail |= (uint32_t)((m & ((c.need >> (i * L.N)) & nmask(L.N))) == 0) << i;
    }
    if (fail & live) return EV_FALSE;
  }
  return EV_TRUE;
}

// DuplicateNullKeyMessage, compaction.tla:280-294 (model.h inv_dupnull)
TLCG_HD int inv_dupnull_k(const Layout& L, const CompMsgs& c, lkey k) {
  const int ctx = k_ctx(L, k);
  if (!(L.retain && ctx != 0)) return EV_TRUE;
  if (ctx > L.C || !k_led_present(L, k, ctx)) return EV_ERROR;
  const int hz = k_hz(L, k);
  const u64 after = nmask(c.len < L.N ? c.len : L.N) & ~nmask(hz);
  return ((u64)k_led_mask(L, k, ctx) & c.null_pos & after) ? EV_FALSE : EV_TRUE;
}

// first failing invariant in cfg order: -1 all hold, else (index << 1) | is_error
TLCG_HD int check_invariants_k(const Layout& L, const CompMsgs& c, lkey k) {
  for (int q = 0; q < L.n_inv; ++q) {
    int r;
    switch (L.inv[q]) {
      case INV_TYPESAFE: r = inv_typesafe_k(L, c, k); break;
      case INV_LEAK: r = inv_leak_k(L, k); break;
      case INV_HORIZON: r = inv_horizon_k(L, c, k); break;
      case INV_DUPNULL: r = inv_dupnull_k(L, c, k); break;
      default:
        r = EV_ERROR;
#ifdef TLCG_USER_INV  // a user invariant on the word msgs | k << (messages' bits)
        if (L.inv[q] >= INV_USER)
          r = tlcg_user_eval(L.inv[q] - INV_USER, UVWord<u64>{L, c.msgs | ((u64)k << (L.msg_sh + L.N * L.mw))});
#endif
    }
    if (r != EV_TRUE) return (q << 1) | (r == EV_ERROR ? 1 : 0);
  }
  return -1;
}

}  // namespace tlcg
