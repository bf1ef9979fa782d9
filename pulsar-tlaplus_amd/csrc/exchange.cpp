// pulsar-tlaplus_amd/csrc/exchange.cpp -- the multi-rank BFS level loop
// (run_ranks) and its two transports, RCCL and local threads (exchange.h).
#include "exchange.h"

#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <thread>
#include <type_traits>

namespace tlcg {

// ---------------------------------------------------------------- RCCL -----

namespace {

// RCCL entry points, resolved once from librccl.so.1 (the library torch's
// nccl backend also loads, so one process shares one copy)
struct Rccl {
  ncclResult_t (*GetUniqueId)(ncclUniqueId*);
  ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int);
  ncclResult_t (*CommInitAll)(ncclComm_t*, int, const int*);
  ncclResult_t (*CommDestroy)(ncclComm_t);
  ncclResult_t (*CommAbort)(ncclComm_t);
  ncclResult_t (*CommGetAsyncError)(ncclComm_t, ncclResult_t*);
  ncclResult_t (*CommCount)(const ncclComm_t, int*);
  ncclResult_t (*AllGather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t);
  ncclResult_t (*AllReduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t);
  ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t);
  ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t);
  ncclResult_t (*GroupStart)();
  ncclResult_t (*GroupEnd)();
  const char* (*GetErrorString)(ncclResult_t);
};

const Rccl* load_rccl(std::string* err) {
  static std::once_flag once;
  static Rccl r;
  static bool ok = false;
  static std::string why;
  std::call_once(once, [] {
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) {
      why = std::string("RCCL not loadable: ") + dlerror();
      return;
    }
    bool all = true;
    auto sym = [&](auto& fn, const char* name) {
      fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
      if (!fn) {
        all = false;
        why = std::string("RCCL lacks ") + name;
      }
    };
    sym(r.GetUniqueId, "ncclGetUniqueId");
    sym(r.CommInitRank, "ncclCommInitRank");
    sym(r.CommInitAll, "ncclCommInitAll");
    sym(r.CommDestroy, "ncclCommDestroy");
    sym(r.CommAbort, "ncclCommAbort");
    sym(r.CommGetAsyncError, "ncclCommGetAsyncError");
    sym(r.CommCount, "ncclCommCount");
    sym(r.AllGather, "ncclAllGather");
    sym(r.AllReduce, "ncclAllReduce");
    sym(r.Send, "ncclSend");
    sym(r.Recv, "ncclRecv");
    sym(r.GroupStart, "ncclGroupStart");
    sym(r.GroupEnd, "ncclGroupEnd");
    sym(r.GetErrorString, "ncclGetErrorString");
    ok = all;
  });
  if (!ok && err) *err = why;
  return ok ? &r : nullptr;
}

double comm_timeout_s() {
  const char* v = std::getenv("TLCG_COMM_TIMEOUT_S");
  const double t = v ? std::atof(v) : 0.0;
  return t > 0 ? t : 600.0;
}

class RcclTransport;

// the RCCL state of one context (tlcg_ctx::comm)
struct CommState {
  ncclComm_t comm = nullptr;
  int rank = 0, world = 1, device = 0;
  hipStream_t stream = nullptr;
  uint64_t* d = nullptr;  // device scratch for counts and reductions
  size_t cap = 0;         // its uint64 capacity
  uint64_t* h = nullptr;  // pinned host mirror
  std::unique_ptr<RcclTransport> t;
};

class RcclTransport : public Transport {
 public:
  explicit RcclTransport(CommState* s) : s_(s) {}
  int rank() const override { return s_->rank; }
  int world() const override { return s_->world; }

  bool allgather_rows(const uint64_t* row, uint64_t* out, std::string* err) override {
    const size_t w = row_width(s_->world);
    hipSetDevice(s_->device);  // (the scratch lives on the rank's device)
    if (!scratch(w + w * (size_t)s_->world, err)) return false;
    std::memcpy(s_->h, row, w * 8);
    if (!hip(hipMemcpyAsync(s_->d, s_->h, w * 8, hipMemcpyHostToDevice, s_->stream), "counts to device", err)) return false;
    if (!nccl(R()->AllGather(s_->d, s_->d + w, w, ncclUint64, s_->comm, s_->stream), "ncclAllGather", err))
      return false;
    if (!hip(hipMemcpyAsync(s_->h + w, s_->d + w, w * (size_t)s_->world * 8, hipMemcpyDeviceToHost, s_->stream),
             "counts to host", err) ||
        !wait(err))
      return false;
    std::memcpy(out, s_->h + w, w * (size_t)s_->world * 8);
    return true;
  }

  bool records(tlcg_ctx* c, const uint64_t* send, const uint64_t* recv, std::string* err, bool wait_done) override {
    uint64_t total = 0;
    for (int r = 0; r < s_->world; ++r)
      if (r != s_->rank) total += recv[r];
    void* inbox = nullptr;
    if (tlcg_inbox(c, total, &inbox) != 0) {
      *err = std::string("tlcg_inbox: ") + tlcg_last_error(c);
      return false;
    }
    if (!nccl(R()->GroupStart(), "ncclGroupStart", err)) return false;
    uint64_t off = 0;
    for (int r = 0; r < s_->world; ++r) {
      if (r == s_->rank) continue;
      if (send[r]) {
        void* p = nullptr;
        uint64_t k = 0;
        tlcg_outbox(c, r, &p, &k);
        if (!nccl(R()->Send(p, (size_t)(2 * send[r]), ncclUint64, r, s_->comm, s_->stream), "ncclSend", err)) {
          R()->GroupEnd();
          return false;
        }
      }
      if (recv[r]) {
        char* dst = static_cast<char*>(inbox) + off * 16;
        if (!nccl(R()->Recv(dst, (size_t)(2 * recv[r]), ncclUint64, r, s_->comm, s_->stream), "ncclRecv", err)) {
          R()->GroupEnd();
          return false;
        }
      }
      off += recv[r];
    }
    // the absorb that follows is ordered on the stream; waiting here puts the
    // records under TLCG_COMM_TIMEOUT_S too (a peer that died mid-exchange
    // aborts the communicator instead of hanging the absorb).
    // Without the wait (the pipelined level) the level's one wait_stream()
    // does the same.
    return nccl(R()->GroupEnd(), "ncclGroupEnd", err) && (!wait_done || wait(err));
  }

  // the one-wait level over RCCL is opt-in (TLCG_PIPELINE=1): no run of more
  // than one RCCL rank has recorded its counts and timeline yet, and its one
  // wait bounds the level's kernels as well as the collective under
  // TLCG_COMM_TIMEOUT_S; the default is the two-step level, whose
  // wait covers the send/recv alone
  bool can_pipeline() const override {
    const char* v = std::getenv("TLCG_PIPELINE");
    return v && !std::strcmp(v, "1");
  }
  bool wait_stream(tlcg_ctx*, std::string* err) override { return wait(err); }

  bool allreduce(uint64_t* v, int n, RedOp op, std::string* err) override {
    if (n <= 0) return true;
    hipSetDevice(s_->device);  // (the scratch lives on the rank's device)
    if (!scratch((size_t)n, err)) return false;
    std::memcpy(s_->h, v, (size_t)n * 8);
    const ncclRedOp_t o = op == RED_SUM ? ncclSum : op == RED_MIN ? ncclMin : ncclMax;
    if (!hip(hipMemcpyAsync(s_->d, s_->h, (size_t)n * 8, hipMemcpyHostToDevice, s_->stream), "to device", err) ||
        !nccl(R()->AllReduce(s_->d, s_->d, (size_t)n, ncclUint64, o, s_->comm, s_->stream), "ncclAllReduce", err) ||
        !hip(hipMemcpyAsync(s_->h, s_->d, (size_t)n * 8, hipMemcpyDeviceToHost, s_->stream), "to host", err) ||
        !wait(err))
      return false;
    std::memcpy(v, s_->h, (size_t)n * 8);
    return true;
  }

 private:
  static const Rccl* R() { return load_rccl(nullptr); }
  bool nccl(ncclResult_t r, const char* what, std::string* err) {
    if (r == ncclSuccess) return true;
    *err = std::string(what) + ": " + R()->GetErrorString(r);
    return false;
  }
  bool hip(hipError_t e, const char* what, std::string* err) {
    if (e == hipSuccess) return true;
    *err = std::string(what) + ": " + hipGetErrorString(e);
    return false;
  }
  bool scratch(size_t n, std::string* err) {
    if (n <= s_->cap) return true;
    hipFree(s_->d);
    hipHostFree(s_->h);
    s_->d = nullptr;
    s_->h = nullptr;
    s_->cap = 0;
    const size_t c = std::max<size_t>(n, 4096);
    if (!hip(hipMalloc(&s_->d, c * 8), "comm scratch", err) || !hip(hipHostMalloc(&s_->h, c * 8), "comm scratch", err))
      return false;
    s_->cap = c;
    return true;
  }
  // the stream's collectives done, or an RCCL error / a timeout (a peer that
  // died): the communicator is aborted rather than waited on forever
  bool wait(std::string* err) {
    const auto t0 = std::chrono::steady_clock::now();
    const double limit = comm_timeout_s();
    for (;;) {
      const hipError_t e = hipStreamQuery(s_->stream);
      if (e == hipSuccess) return true;
      if (e != hipErrorNotReady) return hip(e, "stream", err);
      ncclResult_t ae = ncclSuccess;
      if (R()->CommGetAsyncError(s_->comm, &ae) == ncclSuccess && ae != ncclSuccess && ae != ncclInProgress) {
        *err = std::string("RCCL: ") + R()->GetErrorString(ae);
        R()->CommAbort(s_->comm);
        s_->comm = nullptr;
        return false;
      }
      if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > limit) {
        *err = "RCCL collective timed out (TLCG_COMM_TIMEOUT_S): a peer rank stopped";
        R()->CommAbort(s_->comm);
        s_->comm = nullptr;
        return false;
      }
      // a collective of a few words completes in microseconds: yield while
      // it is young, back off to 20 us sleeps only past 200 us
      if (std::chrono::steady_clock::now() - t0 < std::chrono::microseconds(200)) std::this_thread::yield();
      else std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
  }
  CommState* s_;
};

CommState* new_state(tlcg_ctx* c, int rank, int world) {
  auto* s = new CommState();
  s->rank = rank;
  s->world = world;
  s->device = ctx_device(c);
  s->stream = static_cast<hipStream_t>(tlcg_stream(c));
  s->t.reset(new RcclTransport(s));
  return s;
}

}  // namespace

bool rccl_available(std::string* err) { return load_rccl(err) != nullptr; }

int comm_init(tlcg_ctx* c, const void* id, std::string* err) {
  const Rccl* R = load_rccl(err);
  if (!R) return -30;
  int rank = 0, world = 1;
  ctx_rank_world(c, &rank, &world);
  int prev = 0;
  hipGetDevice(&prev);
  hipSetDevice(ctx_device(c));
  CommState* s = new_state(c, rank, world);
  ncclUniqueId uid;
  std::memcpy(&uid, id, sizeof uid);
  const ncclResult_t r = R->CommInitRank(&s->comm, world, uid, rank);
  hipSetDevice(prev);
  if (r != ncclSuccess) {
    *err = std::string("ncclCommInitRank: ") + R->GetErrorString(r);
    comm_free(s);
    return -31;
  }
  comm_free(ctx_comm(c));
  ctx_comm(c) = s;
  return 0;
}

int comm_init_all(tlcg_ctx* const* ctxs, int n, std::string* err) {
  const Rccl* R = load_rccl(err);
  if (!R) return -30;
  std::vector<int> devs((size_t)n);
  std::vector<ncclComm_t> comms((size_t)n, nullptr);
  for (int r = 0; r < n; ++r) {
    devs[(size_t)r] = ctx_device(ctxs[r]);
    for (int q = 0; q < r; ++q)
      if (devs[(size_t)q] == devs[(size_t)r]) {
        *err = "RCCL needs one device per rank";
        return -32;
      }
  }
  const ncclResult_t res = R->CommInitAll(comms.data(), n, devs.data());
  if (res != ncclSuccess) {
    *err = std::string("ncclCommInitAll: ") + R->GetErrorString(res);
    return -31;
  }
  for (int r = 0; r < n; ++r) {
    CommState* s = new_state(ctxs[r], r, n);
    s->comm = comms[(size_t)r];
    comm_free(ctx_comm(ctxs[r]));
    ctx_comm(ctxs[r]) = s;
  }
  return 0;
}

int comm_size(tlcg_ctx* c) {
  auto* s = static_cast<CommState*>(ctx_comm(c));
  const Rccl* R = load_rccl(nullptr);
  int n = 0;
  if (!s || !s->comm || !R || R->CommCount(s->comm, &n) != ncclSuccess) return 0;
  return n;
}

Transport* comm_transport(tlcg_ctx* c) {
  auto* s = static_cast<CommState*>(ctx_comm(c));
  return s && s->comm ? s->t.get() : nullptr;
}

void comm_free(void* p) {
  auto* s = static_cast<CommState*>(p);
  if (!s) return;
  int prev = 0;
  hipGetDevice(&prev);
  hipSetDevice(s->device);
  if (s->comm) {
    if (s->stream) hipStreamSynchronize(s->stream);
    if (const Rccl* R = load_rccl(nullptr)) R->CommDestroy(s->comm);
  }
  hipFree(s->d);
  hipHostFree(s->h);
  hipSetDevice(prev);
  delete s;
}

// ------------------------------------------------------ local (threads) -----

class LocalTransport;

struct LocalBoard {
  int n = 0;
  bool pull = false;  // every rank on one device (and TLCG_PULL != 0): absorbs read the outboxes in place
  std::vector<tlcg_ctx*> ctxs;
  std::vector<uint64_t> rows;               // n x (n + 1)
  std::vector<std::vector<uint64_t>> red;   // one vector per rank
  std::vector<std::unique_ptr<LocalTransport>> ts;
  std::mutex m;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t phase = 0;
  void barrier() {
    std::unique_lock<std::mutex> l(m);
    const uint64_t p = phase;
    if (++arrived == n) {
      arrived = 0;
      ++phase;
      cv.notify_all();
    } else {
      cv.wait(l, [&] { return phase != p; });
    }
  }
};

class LocalTransport : public Transport {
 public:
  LocalTransport(LocalBoard* b, int r) : b_(b), r_(r) {}
  int rank() const override { return r_; }
  int world() const override { return b_->n; }

  bool allgather_rows(const uint64_t* row, uint64_t* out, std::string*) override {
    const size_t w = row_width(b_->n);
    std::memcpy(&b_->rows[(size_t)r_ * w], row, w * 8);
    b_->barrier();
    std::memcpy(out, b_->rows.data(), w * (size_t)b_->n * 8);
    b_->barrier();  // rows are rewritten only after every rank has read them
    return true;
  }

  // the destination pulls: every source's outbox for this rank, device to
  // device (over xGMI between GPUs), source-rank-major into the inbox
  bool records(tlcg_ctx* c, const uint64_t*, const uint64_t* recv, std::string* err, bool) override {
    uint64_t total = 0;
    for (int s = 0; s < b_->n; ++s)
      if (s != r_) total += recv[s];
    void* inbox = nullptr;
    bool ok = tlcg_inbox(c, total, &inbox) == 0;
    if (!ok) *err = std::string("tlcg_inbox: ") + tlcg_last_error(c);
    const auto stream = static_cast<hipStream_t>(tlcg_stream(c));
    uint64_t off = 0;
    for (int s = 0; s < b_->n && ok; ++s) {
      if (s == r_ || !recv[s]) continue;
      void* p = nullptr;
      uint64_t k = 0;
      tlcg_outbox(b_->ctxs[(size_t)s], r_, &p, &k);
      const hipError_t e = hipMemcpyPeerAsync(static_cast<char*>(inbox) + off * 16, ctx_device(c), p,
                                              ctx_device(b_->ctxs[(size_t)s]), recv[s] * 16, stream);
      if (e != hipSuccess) {
        ok = false;
        *err = std::string("hipMemcpyPeerAsync: ") + hipGetErrorString(e);
      }
      off += recv[s];
    }
    if (ok && hipStreamSynchronize(stream) != hipSuccess) {
      ok = false;
      *err = "record copies failed";
    }
    b_->barrier();  // no source expands (overwriting its outbox) before every copy landed
    return ok;
  }

  bool can_pull() const override { return b_->pull; }
  // every source's records for this rank where the source's row says its
  // outbox lies (its address as of the all-gather: a pipelined source may
  // already be expanding into its other outbox)
  void pull_sources(tlcg_ctx*, const uint64_t* rows, std::vector<const uint64_t*>* p,
                    std::vector<uint64_t>* k) override {
    const int n = b_->n;
    const size_t w = row_width(n);
    p->clear();
    k->clear();
    for (int s = 0; s < n; ++s) {
      const uint64_t* row = rows + (size_t)s * w;
      if (s == r_ || !row[r_]) continue;
      const auto* base = reinterpret_cast<const uint64_t*>((uintptr_t)row[n + 4]);
      p->push_back(base + 2 * (uint64_t)r_ * row[n + 5]);
      k->push_back(row[r_]);
    }
  }
  void pulled() override { b_->barrier(); }
  // pulling ranks need no barrier after the absorb when the outboxes are
  // double-buffered (ctx_absorb_expand)
  bool can_pipeline() const override { return b_->pull; }

  bool allreduce(uint64_t* v, int n, RedOp op, std::string*) override {
    b_->red[(size_t)r_].assign(v, v + n);
    b_->barrier();
    for (int i = 0; i < n; ++i) {
      uint64_t a = b_->red[0][(size_t)i];
      for (int s = 1; s < b_->n; ++s) {
        const uint64_t x = b_->red[(size_t)s][(size_t)i];
        a = op == RED_SUM ? a + x : op == RED_MIN ? std::min(a, x) : std::max(a, x);
      }
      v[i] = a;
    }
    b_->barrier();
    return true;
  }

 private:
  LocalBoard* b_;
  int r_;
};

LocalBoard* local_board_new(tlcg_ctx* const* ctxs, int n) {
  auto* b = new LocalBoard();
  b->n = n;
  b->ctxs.assign(ctxs, ctxs + n);
  b->rows.assign((size_t)n * row_width(n), 0);
  b->red.resize((size_t)n);
  const char* pv = std::getenv("TLCG_PULL");
  b->pull = !(pv && !std::strcmp(pv, "0"));
  for (int r = 1; r < n; ++r) b->pull = b->pull && ctx_device(ctxs[r]) == ctx_device(ctxs[0]);
  for (int r = 0; r < n; ++r) b->ts.emplace_back(new LocalTransport(b, r));
  return b;
}
void local_board_free(LocalBoard* b) { delete b; }
Transport* local_transport(LocalBoard* b, int rank) { return b->ts[(size_t)rank].get(); }

bool Transport::wait_stream(tlcg_ctx* c, std::string* err) {
  const hipError_t e = hipStreamSynchronize(static_cast<hipStream_t>(tlcg_stream(c)));
  if (e == hipSuccess) return true;
  *err = std::string("stream: ") + hipGetErrorString(e);
  return false;
}

// ------------------------------------------------------------ the loop -----

int run_ranks(tlcg_ctx* c, Transport& t, tlcg_stats* st, std::vector<uint64_t>* levels, std::string* err) {
  const int n = t.world(), me = t.rank();
  // a rank's row: its record count per destination, its failure flag, its inbox capacity
  const size_t w = row_width(n);
  bool failed = false;
  std::string local_err;
  auto fail_local = [&](const char* what) {
    if (!failed) local_err = std::string(what) + ": " + tlcg_last_error(c);
    failed = true;
  };
  tlcg_stats s;
  std::memset(&s, 0, sizeof s);
  // TLCG_RANK_TRACE=1: per-phase wall time of this rank's loop on stderr
  const bool trace = std::getenv("TLCG_RANK_TRACE") != nullptr;
  double ph[7] = {0, 0, 0, 0, 0, 0, 0};  // [1..6]: expand, counts, inbox, records, absorb, end_level
  auto clk = [] { return std::chrono::steady_clock::now(); };
  auto tick = [&](int i, std::chrono::steady_clock::time_point& t) {
    const auto n2 = clk();
    ph[i] += std::chrono::duration<double>(n2 - t).count();
    t = n2;
  };
  int nlev = 0;
  if (tlcg_partition_closed(c) == 1) {
    // no successor leaves its rank: each runs alone; only results are combined
    if (tlcg_run(c, &s) != 0) fail_local("tlcg_run");
  } else {
    if (tlcg_init(c, &s) != 0) fail_local("tlcg_init");
    // Producer modelled: tlcg_init ran this rank's subtrees of the component
    // tree to the end (tree.h, no exchange) unless one raised an error to
    // report or did not fit; then every rank redoes the model on the global
    // engine with the exchange below, which reports TLC's first error
    uint64_t tree[2] = {!failed && ctx_engine(c) == TLCG_ENGINE_TREE ? 1u : 0u, failed ? 1u : 0u};
    if (!t.allreduce(tree, 2, RED_SUM, err)) return -20;
    const bool all_tree = !tree[1] && tree[0] == (uint64_t)n;
    if (!all_tree && !failed && ctx_engine(c) == TLCG_ENGINE_TREE) {
      ctx_disable_tree(c);
      if (tlcg_init(c, &s) != 0) fail_local("tlcg_init");
    }
    std::vector<uint64_t> row(w), rows(w * (size_t)n), send((size_t)n), recv((size_t)n);
    // one host synchronization per level (ctx_absorb_expand) when both the
    // transport and the level's kernels allow it; every rank decides alike
    const bool pipe = !all_tree && t.can_pipeline() && ctx_pipeline_ok(c);
    bool have = false;  // pipe: this rank's next level is already expanded
    for (; !all_tree;) {
      auto tp = clk();
      // expand this rank's newest level (an empty one too: every rank takes
      // part in every level), then ONE collective: the counts all-gather,
      // whose rows also carry each rank's expanded level size, error flag and
      // failure flag.  When the rows say the search is over (every level
      // empty, an error, a failure), the expand is undone -- its level is
      // never absorbed -- so the counts are those of the level loop that
      // decided first (round 3 ran a separate all-reduce before each expand).
      // Pipelined, the expand after the first level's happened inside the
      // previous iteration's ctx_absorb_expand.
      const uint64_t level = failed ? 0 : s.frontier;
      const bool erred = !failed && s.status >= TLCG_VIOLATION;
      const bool live = !failed && s.status == TLCG_RUNNING;
      if (live && !have && tlcg_expand(c, &s) != 0) fail_local("tlcg_expand");
      have = false;
      tick(1, tp);
      for (int d = 0; d < n; ++d) {
        uint64_t k = 0;
        if (live && !failed && d != me) tlcg_outbox(c, d, nullptr, &k);
        row[(size_t)d] = send[(size_t)d] = k;
      }
      row[(size_t)n] = failed ? 1 : 0;
      row[(size_t)n + 1] = t.can_pull() ? ~0ull : ctx_inbox_cap(c);  // (no inbox when pulling)
      row[(size_t)n + 2] = level;
      row[(size_t)n + 3] = erred ? 1 : 0;
      ctx_outbox(c, &row[(size_t)n + 4], &row[(size_t)n + 5]);
      if (!t.allgather_rows(row.data(), rows.data(), err)) return -20;
      tick(2, tp);
      bool any = false, grow = false, stop = false;
      uint64_t levels_total = 0;
      for (int q = 0; q < n; ++q) {
        any |= rows[(size_t)q * w + (size_t)n] != 0;
        stop |= rows[(size_t)q * w + (size_t)n + 3] != 0;
        levels_total += rows[(size_t)q * w + (size_t)n + 2];
        recv[(size_t)q] = q == me ? 0 : rows[(size_t)q * w + (size_t)me];
        uint64_t into_q = 0;  // what rank q receives, against its inbox
        for (int p = 0; p < n; ++p)
          if (p != q) into_q += rows[(size_t)p * w + (size_t)q];
        grow |= into_q > rows[(size_t)q * w + (size_t)n + 1];
      }
      if (any || stop || !levels_total) {
        if (live && !failed) ctx_undo_expand(c, &s);
        break;
      }
      ++nlev;
      uint64_t total = 0;
      for (uint64_t x : recv) total += x;
      if (grow) {
        // an inbox must grow before any record moves: every rank learns
        // whether the allocations held (the rows told all of them to wait)
        if (tlcg_inbox(c, total, nullptr) != 0) fail_local("tlcg_inbox");
        uint64_t bad = failed ? 1 : 0;
        if (!t.allreduce(&bad, 1, RED_SUM, err)) return -20;
        if (bad) break;
      }
      tick(3, tp);
      std::vector<const uint64_t*> src;
      std::vector<uint64_t> cnt;
      if (t.can_pull()) {
        // the sources' outboxes read in place, where their rows say they lie
        t.pull_sources(c, rows.data(), &src, &cnt);
      } else {
        std::string rerr;
        const bool moved = t.records(c, send.data(), recv.data(), &rerr, !pipe);
        if (!moved) {  // (local failure: the transport's collective itself completed)
          failed = true;
          local_err = rerr;
          continue;
        }
        void* in = nullptr;
        tlcg_inbox(c, 0, &in);
        src.push_back(static_cast<const uint64_t*>(in));
        cnt.push_back(total);
      }
      tick(4, tp);
      if (pipe) {
        // absorb, end of level and the next level's expand, one wait; the
        // outboxes are double-buffered, so no rank waits for the others here
        if (!failed && ctx_absorb_expand(c, src.data(), cnt.data(), (int)src.size(), t, &s) != 0)
          fail_local("absorb + expand");
        have = !failed && s.status == TLCG_RUNNING;
        tick(5, tp);
        continue;
      }
      if (!failed && ctx_absorb_from(c, src.data(), cnt.data(), (int)src.size(), &s) != 0) fail_local("absorb");
      // every rank passes pulled() (a failed one too), so no outbox is
      // overwritten while another rank reads it
      if (t.can_pull()) t.pulled();
      tick(5, tp);
      if (!failed && tlcg_end_level(c, &s) != 0) fail_local("tlcg_end_level");
      tick(6, tp);
    }
  }
  if (trace)
    std::fprintf(stderr,
                 "rank %d: %d levels (%llu redone), wall s: expand %.3f counts %.3f inbox %.3f records %.3f "
                 "absorb %.3f end %.3f; device ms: kernels %.1f expand %.1f\n",
                 me, nlev, (unsigned long long)s.levels_redone, ph[1], ph[2], ph[3], ph[4], ph[5], ph[6],
                 s.kernel_ms, s.expand_ms);
  // ---- combine, like one context's level loop would report ----
  std::vector<uint64_t> mine(1u << 16), gen(1u << 16);
  int32_t k = 0, kg = 0;
  if (!failed && tlcg_level_sizes(c, mine.data(), (int32_t)mine.size(), &k) != 0) fail_local("tlcg_level_sizes");
  if (!failed && tlcg_level_generated(c, gen.data(), (int32_t)gen.size(), &kg) != 0)
    fail_local("tlcg_level_generated");
  uint64_t fl = failed ? 1 : 0;
  if (!t.allreduce(&fl, 1, RED_SUM, err)) return -20;
  if (fl) {
    *err = failed ? local_err : "another rank failed";
    return -21;
  }
  k = std::min<int32_t>(k, (int32_t)mine.size());
  kg = std::min<int32_t>(kg, (int32_t)gen.size());
  // the first error: lowest level, then lowest rank
  const uint64_t none = ~0ull;
  uint64_t key = s.status >= TLCG_VIOLATION ? ((uint64_t)s.depth << 16) | (uint64_t)me : none;
  if (!t.allreduce(&key, 1, RED_MIN, err)) return -20;
  const int first = key == none ? -1 : (int)(key & 0xFFFF);
  const size_t cut = key == none ? ~(size_t)0 : (size_t)(key >> 16);  // levels 0..E kept
  const size_t kk = std::min<size_t>((size_t)k, cut);
  uint64_t len = kk;
  if (!t.allreduce(&len, 1, RED_MAX, err)) return -20;
  std::vector<uint64_t> lv(std::max<uint64_t>(len, 1), 0);
  for (size_t i = 0; i < kk; ++i) lv[i] = mine[i];
  if (!t.allreduce(lv.data(), (int)lv.size(), RED_SUM, err)) return -20;
  uint64_t g = 0;
  for (size_t i = 0; i < std::min<size_t>((size_t)kg, cut); ++i) g += gen[i];
  const bool mine_first = first == me;
  uint64_t info[8] = {g,
                      mine_first ? (uint64_t)s.status : 0,
                      mine_first ? (uint64_t)(s.invariant + 1) : 0,
                      mine_first ? (uint64_t)(s.action + 1) : 0,
                      mine_first && s.event_gidx != ~0ull ? s.event_gidx + 1 : 0,
                      s.levels_redone,
                      s.host_states,
                      s.fpset_host_states};
  uint64_t times[2] = {(uint64_t)(s.kernel_ms * 1e6), (uint64_t)(s.expand_ms * 1e6)};  // ns
  if (!t.allreduce(info, 8, RED_SUM, err) || !t.allreduce(times, 2, RED_MAX, err)) return -20;
  while (!lv.empty() && !lv.back()) lv.pop_back();
  tlcg_stats out = s;
  out.generated = info[0];
  out.distinct = 0;
  for (uint64_t x : lv) out.distinct += x;
  out.frontier = first < 0 || lv.empty() ? 0 : lv.back();
  // (an open partition's ranks keep empty levels, tlcg_end_level: the
  // erroring rank's level count may hold an empty last level, which one
  // context would not have pushed -- the summed sizes decide)
  out.depth = (int32_t)lv.size();
  out.status = first < 0 ? TLCG_DONE : (int32_t)info[1];
  out.invariant = (int32_t)info[2] - 1;
  out.action = (int32_t)info[3] - 1;
  out.event_gidx = info[4] ? info[4] - 1 : ~0ull;
  out.levels_redone = info[5];
  out.host_states = info[6];
  out.fpset_host_states = info[7];
  out.kernel_ms = (double)times[0] * 1e-6;
  out.expand_ms = (double)times[1] * 1e-6;
  const double d = (double)out.distinct, gg = (double)out.generated;
  out.fp_collision_optimistic = d * (gg - d) / 18446744073709551616.0;
  out.transport = comm_transport(c) == &t ? 2 : 1;
  // the counterexample, walked across the ranks' stores: every rank can then
  // return it (tlcg_trace_words) without a re-run on one GPU
  if (first >= 0 && !trace_ranks(c, t, first, err)) return -20;
  *st = out;
  if (levels) *levels = lv;
  return 0;
}

}  // namespace tlcg

// ------------------------------------------------------------- C ABI -----

extern "C" {

int tlcg_comm_available(void) { return tlcg::rccl_available(nullptr) ? 1 : 0; }

int tlcg_comm_unique_id(void* id, int32_t cap) {
  const tlcg::Rccl* R = tlcg::load_rccl(nullptr);
  if (!R || !id || cap < (int32_t)sizeof(ncclUniqueId)) return -1;
  ncclUniqueId uid;
  if (R->GetUniqueId(&uid) != ncclSuccess) return -2;
  std::memcpy(id, &uid, sizeof uid);
  return (int)sizeof uid;
}

int tlcg_comm_init(tlcg_ctx* c, const void* id, int32_t len) {
  if (!c || !id || len != (int32_t)sizeof(ncclUniqueId)) return -1;
  std::string err;
  const int r = tlcg::comm_init(c, id, &err);
  if (r) tlcg::ctx_set_error(c, err);
  return r;
}

int tlcg_comm_size(tlcg_ctx* c) { return c ? tlcg::comm_size(c) : 0; }

int tlcg_run_comm(tlcg_ctx* c, tlcg_stats* st, uint64_t* levels, int32_t cap, int32_t* n_levels) {
  if (!c || !st) return -1;
  tlcg::Transport* t = tlcg::comm_transport(c);
  if (!t) {
    tlcg::ctx_set_error(c, "tlcg_run_comm: no communicator (tlcg_comm_init)");
    return -1;
  }
  std::vector<uint64_t> lv;
  std::string err;
  const int r = tlcg::run_ranks(c, *t, st, &lv, &err);
  if (r) {
    tlcg::ctx_set_error(c, err);
    return r;
  }
  if (n_levels) *n_levels = (int32_t)lv.size();
  for (size_t i = 0; levels && i < lv.size() && (int32_t)i < cap; ++i) levels[i] = lv[i];
  return 0;
}

}  // extern "C"
