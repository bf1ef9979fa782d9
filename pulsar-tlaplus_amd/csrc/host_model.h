// pulsar-tlaplus_amd/csrc/host_model.h -- host-side model plumbing shared by
// the runtime: constants -> packed Layout, ASSUME check, TLC value printing.
#pragma once
#include <string>
#include <vector>

#include <memory>

#include "model.h"
#include "tlcgpu.h"
#include "user_inv.h"

namespace tlcg {

struct HostModel {
  Layout L;
  std::vector<int64_t> keyset;    // KeySet = KeySpace \cup {0}, sorted (index = packed key index)
  std::vector<int64_t> valueset;  // ValueSet = ValueSpace \cup {0}, sorted
  u64 n_init;                     // number of initial states
  int max_new_per_state;          // upper bound on distinct successors of one state
  std::shared_ptr<UserProg> user;  // the user invariants' program (user_inv.h), or null
  std::string user_defs;          // their text (tlcg_model.user_defs)
};

// Compiles the user invariants `names` (definitions of m.user_defs) into *P
// (user_inv.cpp); false with a message otherwise.
bool compile_user_invariants(const tlcg_model& m, const HostModel& hm, const std::vector<std::string>& names,
                             UserProg* P, std::string* err);
std::vector<std::string> user_def_names(const char* text);
// The compiled user invariants as device code for the run-time specialized
// kernels (user_inv.cpp; model.h tlcg_user_eval), one function per invariant.
// With the layout: the per-component outcome tables of the invariants that
// read few code bits (component_code.h code_consts_user).
std::string user_device_source(const UserProg& P, const Layout& L);
// what user invariant k's program reads: the state fields (component_code.h
// UserField), the component constants (user_inv.cpp UserConstRead), and its
// host-made outcome table for one class (Len, ledger content mask) over the
// code bits `mask` (2 bits per pattern, 3 = the program decides)
uint32_t user_fields(const UserProg& P, int k);
uint32_t user_const_reads(const UserProg& P, int k);
// (P with its dead instructions replaced by loads of 0: user_static_table's input)
UserProg user_prune_dead(const UserProg& P);
u64 user_static_table(const UserProg& P, const Layout& L, int k, uint32_t mask, int len, uint32_t cm);

// The FPSet slot-hash multiplier (multiply-shift over a T-slot table, linear
// probing) with the fewest probe-loop trips on the insert sequence of the
// first component's BFS in component codes.  Without a Producer every
// component has the same code graph (component_code.h), so the choice holds
// for all of them; the FPSet stays exact for any multiplier.  `group` lanes
// insert together and wait for the longest probe (1: a lane of the component
// engine per component; 16: a component of the tree's closed mode).
uint32_t tune_slot_mult(const HostModel& hm, int T, int group, int candidates);

// the tree's closed mode: a displacement per bucket of component 0's codes
// (bucket (code * *dmult) >> 24, TREE_DISP = 256 buckets), chosen so that
// slot(code) = (multiply-shift slot of `mult` + disp[bucket]) mod T places
// every code of the component in a slot of its own -- a perfect hash for the
// code set every component shares without a Producer, so each insert finds
// its slot at the first probe.  Linear probing stays behind it: the FPSet is
// exact for any table (all zero: the plain multiply-shift slot).  False when
// no table was found (then `disp` is all zero).
bool build_slot_disp(const HostModel& hm, int T, uint32_t mult, uint32_t* dmult, uint16_t* disp);
// the tree's closed mode with the bitmap FPSet (tree_body.h BITS): owner[s] =
// the code of component 0's code set in slot s + 1 (0: none), T entries, under
// the slot of build_slot_disp's (mult, dmult, disp); false unless every code
// of the set has a slot of its own (then the bitmap pass is not used)
bool build_slot_owner(const HostModel& hm, int T, uint32_t mult, uint32_t dmult, const uint16_t* disp,
                      uint32_t* owner);

// the per-lane bitmap pass (component_lane.h): a 24-bit multiplier under
// which lane_slot (the top 8 bits of code x mult) is injective on component
// 0's code set -- without a Producer the code set every component shares --
// and owner[s] = the code in slot s + 1 (0: none), LANE_T entries.  The first
// multiplier of a fixed sequence that works; false when the component has 63
// or more states (the pass's capacity) or no multiplier was found
bool build_lane_phash(const HostModel& hm, uint32_t* mult, uint32_t* owner);
// the per-lane pass's FIFO ring entries (component_lane.h LANE_R, a hipRTC
// define): the smallest power of 2 >= 8 whose ring holds component 0's widest
// queue (the kernel sends a component on to the cascade once tail - head >
// R - 2 after an expansion), 16 when that does not fit or the model has no
// per-lane pass.  Depends on the layout alone (component 0's closure).
int lane_ring_entries(const Layout& L);

// every invariant of the cfg, the user's included: -1, else (index << 1) | is_error
template <typename W>
int host_check_all(const HostModel& hm, W s) {
  return hm.user ? check_invariants_all(hm.L, *hm.user, s) : check_invariants(hm.L, s);
}

// Builds the layout; returns false with a TLC-style message on an ASSUME
// failure (compaction.tla:25-35) or on constants this build cannot pack.
bool build_model(const tlcg_model& m, HostModel* out, std::string* err);

// TLC value syntax of a packed state (compaction.tla:57-70 declaration order).
template <typename W>
std::string format_state(const HostModel& hm, W s);

// Successor of `s` at Next ordinal `ord`; returns 1 ok, 0 disabled, 2 eval error.
template <typename W>
int successor_at(const Layout& L, W s, int ord, W* t);

// All successors in Next order; returns count or -1 on an evaluation error.
template <typename W>
int host_successors(const Layout& L, W s, W* out, int* actions, int cap);

// words of the packed state: 1 (<= 63 bits) or 2 (wide layouts, <= 126 bits)
inline int state_words(const Layout& L) { return L.bits <= 63 ? 1 : 2; }
inline u128 join_words(const uint64_t* w, int n) { return n == 1 ? (u128)w[0] : ((u128)w[0] | ((u128)w[1] << 64)); }
inline void split_words(u128 s, uint64_t* w, int n) {
  w[0] = (uint64_t)s;
  if (n > 1) w[1] = (uint64_t)(s >> 64);
}

}  // namespace tlcg
