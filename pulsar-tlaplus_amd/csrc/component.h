// pulsar-tlaplus_amd/csrc/component.h -- the component engine: an exact
// decomposition of the BFS for closed partitions.
//
// When no enabled disjunct can change `messages` (ModelProducer = FALSE:
// compaction.tla:87,100,132,139,145,151,165,182,186,214 all keep it), the
// reachable graph is the disjoint union of one component per initial
// message sequence.  The owner key that spreads states over GPUs (dist.py)
// then spreads them further over wavefront lanes: lane i of a wave owns
// component i of its batch and runs TLC's FIFO BFS on it with an FPSet in
// LDS (no global atomics), writing every state and its parent pointer to the
// HBM state store (coalesced across the 64 lanes).
//
// Order: TLC -workers 1 processes level d in (component, in-component FIFO)
// order, because level 0 is in component (Init enumeration) order and every
// successor stays in its component.  A lane's queue is exactly that FIFO, so
// the event key (level, component, position, action) orders errors like TLC
// and the parent chain is TLC's trace.
#pragma once
#if !defined(__HIPCC_RTC__)
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "model.h"
#endif

namespace tlcg {

constexpr int COMP_MAXLV = 48;  // BFS levels tracked per component (more -> cascade)

struct CompArgs {
  Layout L;
  u64 comp0;                  // first initial-state index (range mode)
  u64 n_comp;                 // components in this launch
  const u64* list;            // explicit initial-state indices (cascade), or null
  u64* store;                 // [batch][K][64] states
  u64* parents;               // parent refs, same layout
  u64 store_base;             // gidx of store[0]
  int msgs_bits;              // bits of `messages` at the bottom of the word
  u64 rank_tag;               // rank << 56, or'ed into parent refs
  unsigned long long* lvl;    // [COMP_MAXLV] per-level distinct counts
  unsigned long long* totals; // [0] generated, [1] distinct
  unsigned long long* event;  // min event key (see make_comp_event)
  u64* ovf_list;               // components that did not fit: initial-state indices
  unsigned long long* ovf_n;
  unsigned long long* outdeg;  // [3] expanded states that discovered 0 / 1 / 2 new states, or null (not counted)
};

// event key: level 8 | initial-state index 36 | queue position 8 | action 4 | kind 2 | index 4
TLCG_HD u64 make_comp_event(int level, u64 comp, int pos, int action, int kind, int index) {
  return ((u64)level << 56) | ((comp & ((1ull << 36) - 1)) << 20) | ((u64)(pos & 255) << 12) |
         ((u64)(action & 15) << 8) | ((u64)kind << 4) | (u64)(index & 15);
}

#if !defined(__HIPCC_RTC__)
// launches the component BFS with on-chip capacity K states per component
// (K = 64, 128 or 255); returns false on a launch error
bool launch_component(const CompArgs& a, int K, hipStream_t stream);
#endif
// store slots a launch of n components needs at capacity K
TLCG_HD u64 component_store_slots(u64 n_comp, int K) { return (n_comp + 63) / 64 * (u64)K * 64; }

}  // namespace tlcg
