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
  const int ndev = std::max(1, tlcg_device_count());
  std::vector<tlcg_ctx*> ctxs((size_t)n, nullptr);
  // the contexts are created and destroyed by one thread per rank, so the
  // ranks' devices allocate and clear their stores and FPSets at once (ranks
  // sharing one GPU serialize there anyway)
  auto destroy_all = [&] {
    std::vector<std::thread> dt;
    for (auto* c : ctxs)
      if (c) dt.emplace_back([c] { tlcg_destroy(c); });
    for (auto& t : dt) t.join();
  };
  tlcg_peer_access(std::min(n, ndev));
  std::vector<int> crc((size_t)n, 0);
  {
    std::vector<std::thread> ct;
    for (int r = 0; r < n; ++r)
      ct.emplace_back([&, r] {
        tlcg_opts o = *base;
        o.device = r % ndev;  // more ranks than devices: ranks share a device
        o.rank = r;
        o.world = n;
        crc[(size_t)r] = tlcg_create(m, &o, &ctxs[(size_t)r]);
      });
    for (auto& t : ct) t.join();
  }
  for (int r = 0; r < n; ++r)
    if (crc[(size_t)r]) {
      put_err(err, err_cap, "tlcg_create (rank " + std::to_string(r) + "): " +
                                (ctxs[(size_t)r] ? tlcg_last_error(ctxs[(size_t)r]) : "no context"));
      const int c = crc[(size_t)r];
      destroy_all();
      return c < 0 ? c : -1;
    }
  const char* force = std::getenv("TLCG_NODE_TRANSPORT");
  std::string why = n > ndev ? "more ranks than devices" : "TLCG_NODE_TRANSPORT=local";
  bool rccl = n <= ndev && !(force && !std::strcmp(force, "local")) && tlcg::rccl_available(&why);
  if (rccl && tlcg::comm_init_all(ctxs.data(), n, &why) != 0) rccl = false;
  if (!rccl && force && !std::strcmp(force, "rccl")) {
    put_err(err, err_cap, "TLCG_NODE_TRANSPORT=rccl: " + why);
    destroy_all();
    return -30;
  }
  tlcg::LocalBoard* board = rccl ? nullptr : tlcg::local_board_new(ctxs.data(), n);
  std::vector<tlcg_stats> sts((size_t)n);
  std::vector<std::vector<uint64_t>> lvs((size_t)n);
  std::vector<std::string> errs((size_t)n);
  std::vector<int> rc((size_t)n, 0);
  std::vector<std::thread> th;
  for (int r = 0; r < n; ++r)
    th.emplace_back([&, r] {
      tlcg::Transport* t = rccl ? tlcg::comm_transport(ctxs[(size_t)r]) : tlcg::local_transport(board, r);
      rc[(size_t)r] = tlcg::run_ranks(ctxs[(size_t)r], *t, &sts[(size_t)r], &lvs[(size_t)r], &errs[(size_t)r]);
    });
  for (auto& t : th) t.join();
  tlcg::local_board_free(board);
  for (int r = 0; r < n; ++r)
    if (rc[(size_t)r]) {
      put_err(err, err_cap, "rank " + std::to_string(r) + ": " + errs[(size_t)r]);
      destroy_all();
      return rc[(size_t)r];
    }
  // every rank holds the combined result
  *st = sts[0];
  st->transport = rccl ? 2 : 1;
  const auto& lv = lvs[0];
  if (levels_out)
    for (size_t i = 0; i < lv.size() && (int32_t)i < cap; ++i) levels_out[i] = lv[i];
  if (n_levels) *n_levels = (int32_t)lv.size();
  // the first error's counterexample, walked across the ranks' stores by
  // run_ranks (every rank holds it)
  if (trace_len && st->status >= TLCG_VIOLATION) {
    int32_t tn = 0;
    if (tlcg_trace_words(ctxs[0], states, actions, trace_cap, &tn) == 0) *trace_len = tn;
  }
  destroy_all();
  return 0;
}
