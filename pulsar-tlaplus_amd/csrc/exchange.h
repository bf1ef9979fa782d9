// pulsar-tlaplus_amd/csrc/exchange.h -- the multi-rank BFS level loop and the
// transports that move its data between ranks (internal to libtlcgpu.so).
//
// One rank = one tlcg_ctx owning a shard of the fingerprint space (SURVEY
// 8(e); TLC's distributed FPSetManager).  run_ranks() is the whole check of
// one rank: a closed partition (no action writes `messages`) runs alone and
// only the results are combined; an open one runs, per BFS level,
//   tlcg_expand -> counts (all-gather, which also carries every rank's
//   termination and error flags: one collective per level) -> records
//   (grouped send/recv of the 16-B {state, parent_ref} outboxes) ->
//   tlcg_absorb -> tlcg_end_level.  Two transports carry it:
//   RcclTransport  -- RCCL over xGMI (one communicator per rank, on the
//                     context's stream; one process per GPU or one thread
//                     per GPU);
//   LocalTransport -- host threads of one process sharing a board, records
//                     copied device to device (ranks that share a GPU).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "tlcgpu.h"

namespace tlcg {

enum RedOp { RED_SUM = 0, RED_MIN = 1, RED_MAX = 2 };

// words of a rank's row in the per-level all-gather: its record count per
// destination, its failure flag, its inbox capacity, the size of the level it
// expanded, its error flag, its outbox's device address and its records per
// destination (run_ranks)
inline size_t row_width(int world) { return (size_t)world + 6; }

class Transport {
 public:
  virtual ~Transport() = default;
  virtual int rank() const = 0;
  virtual int world() const = 0;
  // row[d] = records this rank holds for rank d (row[rank] = 0), row[world] =
  // this rank's failure flag, row[world + 1] its inbox capacity, row[world +
  // 2] the level it expanded, row[world + 3] its error flag; out gets every
  // rank's row (world x row_width(world))
  virtual bool allgather_rows(const uint64_t* row, uint64_t* out, std::string* err) = 0;
  // every outbox of ctx to its owner; the inbox (already sized for the sum of
  // recv) receives them source-rank-major.  Ordered before later work on the
  // context's stream.
  virtual bool records(tlcg_ctx* c, const uint64_t* send, const uint64_t* recv, std::string* err,
                       bool wait = true) = 0;
  virtual bool allreduce(uint64_t* v, int n, RedOp op, std::string* err) = 0;
  // Ranks that share one device need no copy: the destination's absorb reads
  // every source's outbox in place.  can_pull() says this transport does so;
  // pull_sources() gives one {records, count} per source for ctx (recv[s] =
  // the count from rank s); pulled() returns once every rank's absorb is done
  // with the outboxes (no source expands over its outbox before).
  virtual bool can_pull() const { return false; }
  // rows: the level's all-gathered rows (row_width(world) words each, whose
  // words world + 4 / world + 5 hold each rank's outbox address and its
  // records per destination)
  virtual void pull_sources(tlcg_ctx*, const uint64_t* /*rows*/, std::vector<const uint64_t*>*,
                            std::vector<uint64_t>*) {}
  virtual void pulled() {}
  // The one-synchronization level (ctx_absorb_expand): the transport moves
  // a level's records without waiting for them (records(..., wait = false))
  // and wait_stream() is the level's one wait on the context's stream.
  virtual bool can_pipeline() const { return false; }
  virtual bool wait_stream(tlcg_ctx* c, std::string* err);
};

// The check of one rank; *st, levels and the return value are the combined
// result of all ranks (the same on every rank).  0 ok, < 0 error (err).
int run_ranks(tlcg_ctx* c, Transport& t, tlcg_stats* st, std::vector<uint64_t>* levels, std::string* err);

// RCCL (loaded at run time from librccl.so.1, the ROCm collective library).
bool rccl_available(std::string* err);
// a communicator for c (rank and world from its options) from a 128-byte id
int comm_init(tlcg_ctx* c, const void* id, std::string* err);
// one communicator per context, all devices distinct, one process (ncclCommInitAll)
int comm_init_all(tlcg_ctx* const* ctxs, int n, std::string* err);
Transport* comm_transport(tlcg_ctx* c);  // the context's RCCL transport, or null
int comm_size(tlcg_ctx* c);              // ncclCommCount of the context's communicator, 0 if none
void comm_free(void* comm_state);

// the first error's counterexample walked across the ranks' stores (tlcgpu.hip;
// collective over t, after run_ranks has combined the result)
bool trace_ranks(tlcg_ctx* c, Transport& t, int first, std::string* err);

// context internals exchange.cpp needs (tlcgpu.hip)
int ctx_device(const tlcg_ctx* c);
int ctx_engine(const tlcg_ctx* c);         // TLCG_ENGINE_* of the last tlcg_init
uint64_t ctx_inbox_cap(const tlcg_ctx* c); // records the inbox holds without growing
void ctx_disable_tree(tlcg_ctx* c);        // the next tlcg_init runs the global engine
void ctx_rank_world(const tlcg_ctx* c, int* rank, int* world);
void*& ctx_comm(tlcg_ctx* c);
void ctx_set_error(tlcg_ctx* c, const std::string& e);
// forget the last tlcg_expand (its level is never absorbed: the loop ends):
// the generated counts and the pending states as before it; fresh stats
void ctx_undo_expand(tlcg_ctx* c, tlcg_stats* st);
// tlcg_absorb of the records of n sources read where they lie (device memory
// of the context's device): records[i] holds counts[i] {state, parent_ref}
// records.  The local transport's pull: the other ranks' outboxes, no copy.
int ctx_absorb_from(tlcg_ctx* c, const uint64_t* const* records, const uint64_t* counts, int n, tlcg_stats* st);
// the same absorb, then tlcg_end_level, then (the search going on) the next
// level's tlcg_expand, with one wait on the stream (t.wait_stream) when
// ctx_pipeline_ok(c); the records must be readable in stream order
int ctx_absorb_expand(tlcg_ctx* c, const uint64_t* const* records, const uint64_t* counts, int n, Transport& t,
                      tlcg_stats* st);
bool ctx_pipeline_ok(const tlcg_ctx* c);
// device address of c's current outbox and its records per destination
void ctx_outbox(const tlcg_ctx* c, uint64_t* addr, uint64_t* per_dst);

// The local transport of n ranks driven by n threads of this process.
struct LocalBoard;
LocalBoard* local_board_new(tlcg_ctx* const* ctxs, int n);
void local_board_free(LocalBoard* b);
Transport* local_transport(LocalBoard* b, int rank);  // owned by the board

}  // namespace tlcg
