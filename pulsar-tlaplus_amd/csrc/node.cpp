// pulsar-tlaplus_amd/csrc/node.cpp -- tlcg_run_node: one process checks the
// model on every GPU of a node, one context (rank) per device, the FPSet
// hash-partitioned by owner, each rank driven by its own host thread.  This is
// what `tlc-hip -gpus N` runs; the one-process-per-GPU form is tlcg_comm_init +
// tlcg_run_comm (python/dist.py run_native).  Both run the same level loop,
// exchange.cpp run_ranks():
//
//   closed partition (no Producer: `messages` is immutable, so successors never
//     leave their rank, compaction.tla:87,100,132,139,145,151,165,182,186,214):
//     every rank runs tlcg_run to completion, then the results are combined;
//   open partition (Producer, or tlcg_opts.partition = 2): every level is
//     tlcg_expand -> counts all-gather -> records send/recv to their owners ->
//     tlcg_absorb + tlcg_end_level, until a rank stops or no rank found a new
//     state.
//
// Transport: RCCL over xGMI (ncclCommInitAll, one communicator per device)
// when every rank has a device of its own; otherwise (more ranks than
// devices) host threads meeting at a board, records copied device to device.
// TLCG_NODE_TRANSPORT=local|rccl forces one.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "exchange.h"
#include "tlcgpu.h"

namespace {

void put_err(char* err, int32_t cap, const std::string& s) {
  if (err && cap > 0) std::snprintf(err, (size_t)cap, "%s", s.c_str());
}

}  // namespace

// The ranks of one node, kept across checks (tlcg_node_*): every rank's
// context -- its FPSet shard, store, outboxes and inbox, sized by the first
// check -- and the transport between them.  A check then costs its level
// loop only; creating and freeing eight contexts (each with its GiB-sized
// FPSet shard) took 0.06-2.7 s of host time per check when every call of
// tlcg_run_node built them anew (profiles/r03_node8_g9_v9.jsonl).
struct tlcg_node {
  int n = 0;
  bool rccl = false;
  std::vector<tlcg_ctx*> ctxs;
  tlcg::LocalBoard* board = nullptr;
};

namespace {

void destroy_ctxs(std::vector<tlcg_ctx*>& ctxs) {
  // one thread per rank, so the ranks' devices free at once
  std::vector<std::thread> dt;
  for (auto* c : ctxs)
    if (c) dt.emplace_back([c] { tlcg_destroy(c); });
  for (auto& t : dt) t.join();
  for (auto*& c : ctxs) c = nullptr;
}

}  // namespace

extern "C" int tlcg_node_create(const tlcg_model* m, const tlcg_opts* base, int32_t n, tlcg_node** out, char* err,
                                int32_t err_cap) {
  if (out) *out = nullptr;
  if (!m || !base || !out || n < 1 || n > 64) {
    put_err(err, err_cap, "tlcg_node_create: bad arguments");
    return -1;
  }
  const int ndev = std::max(1, tlcg_device_count());
  auto* node = new tlcg_node();
  node->n = n;
  node->ctxs.assign((size_t)n, nullptr);
  tlcg_peer_access(std::min(n, ndev));
  std::vector<int> crc((size_t)n, 0);
  {
    // one thread per rank: the ranks' devices allocate and clear their stores
    // and FPSets at once (ranks sharing one GPU serialize there anyway)
    std::vector<std::thread> ct;
    for (int r = 0; r < n; ++r)
      ct.emplace_back([&, r] {
        tlcg_opts o = *base;
        o.device = r % ndev;  // more ranks than devices: ranks share a device
        o.rank = r;
        o.world = n;
        crc[(size_t)r] = tlcg_create(m, &o, &node->ctxs[(size_t)r]);
      });
    for (auto& t : ct) t.join();
  }
  for (int r = 0; r < n; ++r)
    if (crc[(size_t)r]) {
      put_err(err, err_cap, "tlcg_create (rank " + std::to_string(r) + "): " +
                                (node->ctxs[(size_t)r] ? tlcg_last_error(node->ctxs[(size_t)r]) : "no context"));
      const int c = crc[(size_t)r];
      tlcg_node_destroy(node);
      return c < 0 ? c : -1;
    }
  const char* force = std::getenv("TLCG_NODE_TRANSPORT");
  std::string why = n > ndev ? "more ranks than devices" : "TLCG_NODE_TRANSPORT=local";
  node->rccl = n <= ndev && !(force && !std::strcmp(force, "local")) && tlcg::rccl_available(&why);
  if (node->rccl && tlcg::comm_init_all(node->ctxs.data(), n, &why) != 0) node->rccl = false;
  if (!node->rccl && force && !std::strcmp(force, "rccl")) {
    put_err(err, err_cap, "TLCG_NODE_TRANSPORT=rccl: " + why);
    tlcg_node_destroy(node);
    return -30;
  }
  if (!node->rccl) node->board = tlcg::local_board_new(node->ctxs.data(), n);
  *out = node;
  return 0;
}

extern "C" int tlcg_node_run(tlcg_node* node, tlcg_stats* st, uint64_t* levels_out, int32_t cap, int32_t* n_levels,
                             uint64_t* states, int32_t* actions, int32_t trace_cap, int32_t* trace_len, char* err,
                             int32_t err_cap) {
  if (trace_len) *trace_len = 0;
  if (!node || !st) {
    put_err(err, err_cap, "tlcg_node_run: bad arguments");
    return -1;
  }
  const int n = node->n;
  std::vector<tlcg_stats> sts((size_t)n);
  std::vector<std::vector<uint64_t>> lvs((size_t)n);
  std::vector<std::string> errs((size_t)n);
  std::vector<int> rc((size_t)n, 0);
  std::vector<std::thread> th;
  for (int r = 0; r < n; ++r)
    th.emplace_back([&, r] {
      tlcg_ctx* c = node->ctxs[(size_t)r];
      tlcg::Transport* t = node->rccl ? tlcg::comm_transport(c) : tlcg::local_transport(node->board, r);
      if (!t) {
        rc[(size_t)r] = -20;
        errs[(size_t)r] = "no transport (a communicator was aborted by an earlier check)";
        return;
      }
      rc[(size_t)r] = tlcg::run_ranks(c, *t, &sts[(size_t)r], &lvs[(size_t)r], &errs[(size_t)r]);
    });
  for (auto& t : th) t.join();
  for (int r = 0; r < n; ++r)
    if (rc[(size_t)r]) {
      put_err(err, err_cap, "rank " + std::to_string(r) + ": " + errs[(size_t)r]);
      return rc[(size_t)r];
    }
  // every rank holds the combined result
  *st = sts[0];
  st->transport = node->rccl ? 2 : 1;
  const auto& lv = lvs[0];
  if (levels_out)
    for (size_t i = 0; i < lv.size() && (int32_t)i < cap; ++i) levels_out[i] = lv[i];
  if (n_levels) *n_levels = (int32_t)lv.size();
  // the first error's counterexample, walked across the ranks' stores by
  // run_ranks (every rank holds it)
  if (trace_len && st->status >= TLCG_VIOLATION) {
    int32_t tn = 0;
    if (tlcg_trace_words(node->ctxs[0], states, actions, trace_cap, &tn) == 0) *trace_len = tn;
  }
  return 0;
}

extern "C" void tlcg_node_destroy(tlcg_node* node) {
  if (!node) return;
  tlcg::local_board_free(node->board);
  destroy_ctxs(node->ctxs);
  delete node;
}

extern "C" int tlcg_run_node(const tlcg_model* m, const tlcg_opts* base, int32_t n, tlcg_stats* st,
                             uint64_t* levels_out, int32_t cap, int32_t* n_levels, char* err, int32_t err_cap) {
  return tlcg_run_node_trace(m, base, n, st, levels_out, cap, n_levels, nullptr, nullptr, 0, nullptr, err, err_cap);
}

extern "C" int tlcg_run_node_trace(const tlcg_model* m, const tlcg_opts* base, int32_t n, tlcg_stats* st,
                                   uint64_t* levels_out, int32_t cap, int32_t* n_levels, uint64_t* states,
                                   int32_t* actions, int32_t trace_cap, int32_t* trace_len, char* err,
                                   int32_t err_cap) {
  if (trace_len) *trace_len = 0;
  if (!m || !base || !st || n < 1 || n > 64) {
    put_err(err, err_cap, "tlcg_run_node: bad arguments");
    return -1;
  }
  tlcg_node* node = nullptr;
  const int r = tlcg_node_create(m, base, n, &node, err, err_cap);
  if (r) return r;
  const int q = tlcg_node_run(node, st, levels_out, cap, n_levels, states, actions, trace_cap, trace_len, err, err_cap);
  tlcg_node_destroy(node);
  return q;
}
