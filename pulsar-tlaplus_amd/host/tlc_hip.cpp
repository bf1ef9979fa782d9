// pulsar-tlaplus_amd/host/tlc_hip.cpp -- `tlc-hip`, the drop-in for
//   java tlc2.TLC [-workers N] [-deadlock] [-config F.cfg] compaction.tla
// on one MI355X.  Parses the cfg, recognizes the module, checks the ASSUME,
// runs the BFS through libtlcgpu.so and prints TLC's report: states
// generated, distinct states, depth, verdict and (on an error) the trace.
#include <sys/stat.h>

#include <algorithm>
#include <cerrno>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <ctime>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "cfg.h"
#include "tlcgpu.h"

using namespace tlchost;

namespace {

const char* kActionName[] = {"Producer", "CompactorPhaseOne", "CompactorPhaseTwoWrite",
                             "CompactorPhaseTwoUpdateContext", "CompactorPhaseTwoUpdateHorizon",
                             "CompactorPhaseTwoPersistCusror", "CompactorPhaseTwoDeleteLedger",
                             "BrokerCrash", "Consumer", "Terminating"};

bool read_file(const std::string& p, std::string* out) {
  std::ifstream f(p, std::ios::binary);
  if (!f) return false;
  std::ostringstream s;
  s << f.rdbuf();
  *out = s.str();
  return true;
}

std::string now_str() {
  std::time_t t = std::time(nullptr);
  char b[64];
  std::strftime(b, sizeof b, "%Y-%m-%d %H:%M:%S", std::localtime(&t));
  return b;
}

std::string duration_str(double secs) {  // TLC's "Finished in" form
  long s = (long)std::floor(secs);
  char b[64];
  if (s < 60) std::snprintf(b, sizeof b, "%02lds", s);
  else if (s < 3600) std::snprintf(b, sizeof b, "%02ldmin %02lds", s / 60, s % 60);
  else std::snprintf(b, sizeof b, "%02ldh %02ldmin", s / 3600, (s % 3600) / 60);
  return b;
}

std::string prob_str(double p) {  // Java-like "3.8E-11"
  if (p <= 0) return "0.0";
  int e = (int)std::floor(std::log10(p));
  double mant = p / std::pow(10.0, e);
  if (mant >= 9.95) { mant /= 10; ++e; }
  char b[64];
  if (e >= -3 && e < 7) std::snprintf(b, sizeof b, "%.1f", p);
  else std::snprintf(b, sizeof b, "%.1fE%d", mant, e);
  return b;
}

void usage() {
  std::fprintf(stderr,
               "usage: tlc-hip [-config FILE.cfg] [-deadlock] [-workers N] [-gpu D | -gpus N] [-fpbits B] [-defs FILE]\n"
               "               [-checkpoint MINUTES] [-metadir DIR] [-recover DIR]\n"
               "               [-tlc-order] [-no-trace] [-json] [-dump-defs] [SPEC.tla]\n"
               "  without SPEC.tla: the built-in compaction module, with -config FILE.cfg\n"
               "  -defs FILE: definitions added to the built-in module (\"Name == expr\" at column 1), e.g.\n"
               "              invariants the cfg names (user invariants: include/tlcgpu.h)\n");
}

struct Opts {
  std::string spec, cfg, metadir, recover;
  bool deadlock_off = false, tlc_order = false, trace = true, json = false, dump_defs = false;
  std::string defs;  // -defs FILE: definitions added to the built-in module (user invariants)
  int gpu = 0, gpus = 1, fpbits = 0;
  double checkpoint_min = 30.0;  // TLC's default interval; 0 = never
};

// TLC's metadir name: states/yy-MM-dd-HH-mm-ss next to the spec
std::string default_metadir(const std::string& spec) {
  std::time_t t = std::time(nullptr);
  char b[64];
  std::strftime(b, sizeof b, "%y-%m-%d-%H-%M-%S", std::localtime(&t));
  const size_t slash = spec.find_last_of('/');
  return (slash == std::string::npos ? std::string() : spec.substr(0, slash + 1)) + "states/" + b;
}

bool make_dirs(const std::string& p) {
  for (size_t i = 1; i <= p.size(); ++i)
    if (i == p.size() || p[i] == '/') {
      const std::string d = p.substr(0, i);
      if (mkdir(d.c_str(), 0755) != 0 && errno != EEXIST) return false;
    }
  return true;
}

const char* kCheckpointFile = "/tlcg.ckpt";

// source extent of an action's definition body, for TLC's "<Action line .. of module ..>"
std::string action_location(const Module& mod, int action) {
  const Def* d = mod.find(kActionName[action]);
  if (!d) return kActionName[action];
  char b[256];
  std::snprintf(b, sizeof b, "%s line %d, col %d to line %d, col %d of module %s", kActionName[action], d->line0,
                d->col0, d->line1, d->col1, mod.name.c_str());
  return b;
}

}  // namespace

int main(int argc, char** argv) {
  Opts o;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto next = [&]() -> std::string { return i + 1 < argc ? argv[++i] : ""; };
    if (a == "-config") o.cfg = next();
    else if (a == "-deadlock") o.deadlock_off = true;
    else if (a == "-workers") next();  // TLC worker threads: the GPU is the worker pool
    else if (a == "-fp" || a == "-seed" || a == "-fpmem") next();
    else if (a == "-metadir") o.metadir = next();
    else if (a == "-recover") o.recover = next();
    else if (a == "-checkpoint") {
      char* end = nullptr;
      const std::string v = next();
      o.checkpoint_min = std::strtod(v.c_str(), &end);
      if (v.empty() || *end || o.checkpoint_min < 0) {
        std::fprintf(stderr, "Error: -checkpoint needs a number of minutes\n");
        return 255;
      }
    }
    else if (a == "-cleanup" || a == "-nowarning" || a == "-terse") {}
    else if (a == "-gpu") o.gpu = std::atoi(next().c_str());
    else if (a == "-gpus") o.gpus = std::atoi(next().c_str());
    else if (a == "-fpbits") o.fpbits = std::atoi(next().c_str());
    else if (a == "-tlc-order") o.tlc_order = true;
    else if (a == "-no-trace") o.trace = false;
    else if (a == "-json") o.json = true;
    else if (a == "-dump-defs") o.dump_defs = true;
    else if (a == "-defs") o.defs = next();
    else if (a == "-h" || a == "-help") { usage(); return 0; }
    else if (!a.empty() && a[0] == '-') { std::fprintf(stderr, "Error: unsupported option %s\n", a.c_str()); usage(); return 255; }
    else o.spec = a;
  }
  // no SPEC.tla: check the built-in module (the definitions of compaction.tla
  // as this build implements them), the cfg given by -config
  const bool builtin = o.spec.empty() && !o.cfg.empty() && !o.dump_defs;
  if (o.spec.empty() && !builtin) { usage(); return 255; }
  if (o.gpus < 1 || o.gpus > 64) { std::fprintf(stderr, "Error: -gpus needs 1..64\n"); return 255; }
  if (o.gpus > 1 && !o.recover.empty()) { std::fprintf(stderr, "Error: -recover runs on one GPU\n"); return 255; }
  if (o.gpus > 1) o.checkpoint_min = 0;  // checkpoints hold one context's levels
  if (builtin) o.spec = "compaction.tla";
  if (o.spec.size() < 4 || o.spec.substr(o.spec.size() - 4) != ".tla") o.spec += ".tla";
  if (o.cfg.empty()) o.cfg = o.spec.substr(0, o.spec.size() - 4) + ".cfg";

  std::string tla, cfgtext, err;
  Module mod;
  if (builtin) {
    mod = builtin_module();
    if (!o.defs.empty()) {
      // definitions added to the built-in module (its .tla text is not at
      // hand, e.g. on a GPU host): "Name == expr" items at column 1
      std::string extra;
      if (!read_file(o.defs, &extra)) { std::printf("Error: cannot read %s\n", o.defs.c_str()); return 255; }
      Module add;
      if (!parse_module("---- MODULE defs ----\n" + extra + "\n====\n", &add, &err)) {
        std::printf("Error: %s\n", err.c_str());
        return 150;
      }
      for (Def d : add.defs) {
        if (d.name == "__DECLARATIONS__" || d.name == "ASSUME") continue;
        d.line0 -= 1;
        d.line1 -= 1;
        auto it = mod.by_name.find(d.name);
        if (it != mod.by_name.end()) mod.defs[it->second] = d;
        else {
          mod.by_name[d.name] = mod.defs.size();
          mod.defs.push_back(d);
        }
      }
    }
  } else {
    if (!read_file(o.spec, &tla)) { std::printf("Error: cannot read %s\n", o.spec.c_str()); return 255; }
    if (!parse_module(tla, &mod, &err)) { std::printf("Error: %s\n", err.c_str()); return 150; }
  }
  if (o.dump_defs) {  // maintenance: fingerprints for known_defs.inc
    for (auto& d : mod.defs) {
      uint64_t h = 1469598103934665603ull;
      for (unsigned char c : d.norm) { h ^= c; h *= 1099511628211ull; }
      std::printf("    {\"%s\", 0x%016llxull, %d, %d, %d, %d},\n", d.name.c_str(), (unsigned long long)h, d.line0,
                  d.col0, d.line1, d.col1);
    }
    return 0;
  }
  auto t0 = std::chrono::steady_clock::now();
  std::printf("tlc-hip: TLC-compatible breadth-first model checking on MI355X (libtlcgpu ABI %d)\n",
              tlcg_abi_version());
  if (o.gpus > 1)
    std::printf("Running breadth-first search Model-Checking with %d GPU ranks (FPSet partitioned by owner, rank r on device r mod %d) and seed 0.\n",
                o.gpus, std::max(1, tlcg_device_count()));
  else
    std::printf("Running breadth-first search Model-Checking with 1 GPU (device %d) and seed 0.\n", o.gpu);
  if (builtin) std::printf("Parsing file %s (built-in: the definitions of compaction.tla this build implements)\n", o.spec.c_str());
  else std::printf("Parsing file %s\n", o.spec.c_str());
  if (!recognize_compaction(mod, &err)) { std::printf("Error: %s\n", err.c_str()); return 150; }
  if (!read_file(o.cfg, &cfgtext)) { std::printf("Error: cannot read configuration file %s\n", o.cfg.c_str()); return 151; }
  Config cfg;
  if (!parse_cfg(cfgtext, &cfg, &err)) { std::printf("Error: %s\n", err.c_str()); return 151; }  // ERROR_CONFIG_PARSE
  std::printf("Semantic processing of module %s\n", mod.name.c_str());
  std::printf("Starting... (%s)\n", now_str().c_str());
  tlcg_model model;
  int code = 0, fairness = TLCG_FAIR_NONE;
  if (!bind_model(cfg, mod, o.deadlock_off, &model, &err, &code, &fairness)) {
    std::printf("%s\n", err.c_str());
    std::printf("Finished in %s at (%s)\n", duration_str(0).c_str(), now_str().c_str());
    return code;
  }
  char cerr[512];
  if (tlcg_check_model(&model, cerr, sizeof cerr) != 0) { std::printf("Error: %s\n", cerr); return 150; }
  const std::string recover_file = o.recover.empty() ? "" : o.recover + kCheckpointFile;
  if (!recover_file.empty()) {
    std::ifstream probe(recover_file, std::ios::binary);
    if (!probe) { std::printf("Error: cannot read checkpoint %s\n", recover_file.c_str()); return 150; }
  }
  if (o.metadir.empty()) o.metadir = default_metadir(o.spec);

  tlcg_opts opts;
  std::memset(&opts, 0, sizeof opts);
  opts.device = o.gpu;
  opts.log2_fpset_slots = o.fpbits;
  opts.tlc_order = o.tlc_order;
  opts.world = 1;
  // like TLC's disk-backed trace and queue: committed levels move to host
  // memory when HBM runs short (never otherwise)
  opts.spill = 1;
  opts.fpset_spill = tlcg_state_words(&model) == 1;  // and TLC's DiskFPSet: the host tier (narrow states)
  opts.outdegree = 1;  // TLC's outdegree line
  if (!recover_file.empty()) opts.engine = TLCG_ENGINE_GLOBAL;  // checkpoints are global-engine level states
  else std::printf("Computing initial states...\n");
  tlcg_ctx* ctx = nullptr;
  tlcg_stats st;
  // -gpus N: the first error's counterexample walked across the ranks' stores
  // (printed when the one-GPU TLC-order re-run below cannot be made)
  const int state_words = tlcg_state_words(&model);
  std::vector<uint64_t> node_states;
  std::vector<int32_t> node_acts;
  int32_t node_tlen = 0;
  if (o.gpus > 1) {
    char merr[512];
    node_states.resize((size_t)state_words << 16);
    node_acts.resize(1 << 16);
    if (tlcg_run_node_trace(&model, &opts, o.gpus, &st, nullptr, 0, nullptr, node_states.data(), node_acts.data(),
                            (int32_t)node_acts.size(), &node_tlen, merr, sizeof merr) != 0) {
      std::printf("Error: %s\n", merr);
      return 255;
    }
    const unsigned long long n0 = (unsigned long long)tlcg_init_count(&model);
    std::printf("Finished computing initial states: %llu distinct state%s generated at %s.\n", n0, n0 == 1 ? "" : "s",
                now_str().c_str());
  } else if (tlcg_create(&model, &opts, &ctx) != 0) {
    std::printf("Error: %s\n", ctx ? tlcg_last_error(ctx) : "tlcg_create failed");
    tlcg_destroy(ctx);
    return 255;
  }
  if (ctx && !recover_file.empty()) {
    // [TLC-ext] TLC's recovery messages
    std::printf("Starting recovery from checkpoint %s\n", o.recover.c_str());
    if (tlcg_recover(ctx, recover_file.c_str(), &st) != 0) {
      std::printf("Error: %s\n", tlcg_last_error(ctx));
      tlcg_destroy(ctx);
      return 150;
    }
    std::printf("Recovery completed. %llu states examined. %llu states on queue.\n",
                (unsigned long long)(st.distinct - st.frontier), (unsigned long long)st.frontier);
  } else if (ctx) {
    if (tlcg_init(ctx, &st) != 0) { std::printf("Error: %s\n", tlcg_last_error(ctx)); tlcg_destroy(ctx); return 255; }
    // (the initial states: the component engine has finished the whole search by now)
    const unsigned long long n0 = (unsigned long long)tlcg_init_count(&model);
    std::printf("Finished computing initial states: %llu distinct state%s generated at %s.\n", n0, n0 == 1 ? "" : "s",
                now_str().c_str());
  }
  auto last_progress = std::chrono::steady_clock::now();
  auto last_checkpoint = last_progress;
  while (st.status == TLCG_RUNNING) {
    if (tlcg_step_level(ctx, &st) != 0) { std::printf("Error: %s\n", tlcg_last_error(ctx)); tlcg_destroy(ctx); return 255; }
    auto now = std::chrono::steady_clock::now();
    if (o.checkpoint_min > 0 && st.status == TLCG_RUNNING &&
        std::chrono::duration<double>(now - last_checkpoint).count() >= 60.0 * o.checkpoint_min) {
      // [TLC-ext] TLC's checkpoint messages; the file holds the committed levels
      std::printf("Checkpointing of run %s\n", o.metadir.c_str());
      if (!make_dirs(o.metadir) || tlcg_checkpoint(ctx, (o.metadir + kCheckpointFile).c_str()) != 0)
        std::printf("Error: checkpoint failed: %s\n", tlcg_last_error(ctx));
      else
        std::printf("Checkpointing completed at (%s)\n", now_str().c_str());
      std::fflush(stdout);
      last_checkpoint = std::chrono::steady_clock::now();
    }
    if (std::chrono::duration<double>(now - last_progress).count() > 60.0) {
      double mins = std::chrono::duration<double>(now - t0).count() / 60.0;
      std::printf("Progress(%d) at %s: %llu states generated (%.0f s/min), %llu distinct states found (%.0f ds/min), %llu states left on queue.\n",
                  st.depth, now_str().c_str(), (unsigned long long)st.generated, st.generated / mins,
                  (unsigned long long)st.distinct, st.distinct / mins, (unsigned long long)st.frontier);
      last_progress = now;
    }
  }
  int rc = 0;
  uint64_t stop_left = ~0ull;  // TLC's "states left on queue" at an error (tlcg_tlc_stop_stats)
  // PROPERTY Termination, checked like TLC after the safety search of the
  // complete state space ([TLC-ext] message text), on the GPU
  // (tlcg_check_termination: the not-P part of the state graph, its stuck
  // states and, under fairness, its cycles)
  bool live_fail = false;
  if (st.status == TLCG_DONE && !cfg.properties.empty()) {
    std::printf("Checking temporal properties for the complete state space with %llu total distinct states at (%s)\n",
                (unsigned long long)st.distinct, now_str().c_str());
    const int words = tlcg_state_words(&model);
    std::vector<uint64_t> lstates((size_t)words << 16);
    std::vector<int32_t> lacts(1 << 16);
    int32_t ln = 0;
    tlcg_liveness lv;
    tlcg_opts lo = opts;
    lo.state_capacity = st.distinct;  // G' is a subset of the reachable states
    lo.log2_fpset_slots = 0;
    char lerr[512] = {0};
    // (the check allocates its own device buffers beside the safety run's,
    // which the outdegree statistics below still read: per state of capacity
    // the store, parent, slot index and stuck flag, 21-29 B, and 2 FPSet slots
    // of 20-28 B each -- 60-85 B; it halves the capacity until they fit and
    // grows it x4 only if G' needs more, liveness.hip)
    if (tlcg_check_termination(&model, &lo, fairness, &lv, lstates.data(), lacts.data(), (int32_t)lacts.size(), &ln,
                               lerr, (int32_t)sizeof lerr) != 0) {
      std::printf("Error: the liveness check failed: %s\n", lerr);
      std::printf("Finished in %s at (%s)\n", duration_str(0).c_str(), now_str().c_str());
      return 255;
    }
    std::printf("Finished checking temporal properties in %s at %s\n", duration_str(lv.wall_ms / 1000.0).c_str(),
                now_str().c_str());
    if (!lv.holds) {
      live_fail = true;
      std::vector<char> buf(1 << 16);
      std::printf("Error: Temporal properties were violated.\n\n");
      std::printf("Error: The following behavior constitutes a counter-example:\n\n");
      for (int i = 0; i < ln; ++i) {
        if (lacts[(size_t)i] < 0) std::printf("State %d: <Initial predicate>\n", i + 1);
        else std::printf("State %d: <%s>\n", i + 1, action_location(mod, lacts[(size_t)i]).c_str());
        tlcg_decode_words(&model, &lstates[(size_t)i * words], buf.data(), (int32_t)buf.size());
        std::printf("%s\n\n", buf.data());
      }
      if (lv.loop_to < 0) std::printf("State %d: Stuttering\n", ln + 1);
      else std::printf("State %d: Back to state %d: <%s>\n", ln + 1, lv.loop_to + 1,
                       action_location(mod, lv.back_action).c_str());
    }
  }
  if (live_fail) {
    rc = 13;
  } else if (st.status == TLCG_DONE) {
    std::printf("Model checking completed. No error has been found.\n");
    std::printf("  Estimates of the probability that TLC did not check all reachable states\n");
    std::printf("  because two distinct states had the same fingerprint:\n");
    std::printf("  calculated (optimistic):  val = %s\n", prob_str(st.fp_collision_optimistic).c_str());
    std::printf("  (tlc-hip keeps the packed states themselves: its FPSet is exact, actual collision probability 0)\n");
  } else {
    // TLC prints the trace of the first error in its (one-worker) order: reproduce it
    tlcg_ctx* tctx = ctx;
    tlcg_stats tst = st;
    bool own = false, use_node_trace = false;
    // (after -gpus N: on one GPU).  The global engine in TLC order stores the
    // states in TLC's FIFO order, which also gives TLC's statistics at the stop;
    // no re-run when the first run's trace and stop statistics already are
    // TLC's (st.tlc_exact: the component engine's error on one GPU, a TLC-order run)
    if (o.trace && !(ctx && st.tlc_exact) && (!o.tlc_order || !ctx || st.engine != TLCG_ENGINE_GLOBAL)) {
      tlcg_opts to = opts;
      to.tlc_order = 1;
      to.engine = TLCG_ENGINE_GLOBAL;
      if (!ctx) to.device = 0;
      // the first run's device memory is released before the re-run, which
      // needs as much again (and more: TLC order keeps discovery keys)
      tlcg_destroy(ctx);
      ctx = nullptr;
      tctx = nullptr;
      std::string why;
      if (tlcg_create(&model, &to, &tctx) == 0 && tlcg_run(tctx, &tst) == 0 && tst.status == st.status) {
        own = true;
      } else {
        why = tctx ? tlcg_last_error(tctx) : "tlcg_create failed";
        tlcg_destroy(tctx);
        tctx = nullptr;
        tst = st;
        // fall back to the first run's engine and order: a shortest
        // counterexample, but not necessarily the one TLC -workers 1 prints
        // (-gpus N: the one walked across the ranks' stores, no re-run)
        if (o.gpus > 1 && node_tlen > 0) {
          use_node_trace = true;
          std::printf("Warning: the TLC-order re-run for the trace failed (%s); the trace below is a shortest "
                      "counterexample (walked across the GPUs' stores) but may not be the one TLC prints, and the "
                      "counts are at the end of the level.\n", why.c_str());
        }
        tlcg_opts fo = opts;
        if (!o.recover.empty() || o.gpus > 1) fo.engine = TLCG_ENGINE_GLOBAL;
        tlcg_stats fst;
        if (use_node_trace) {
        } else if (tlcg_create(&model, &fo, &tctx) == 0 && tlcg_run(tctx, &fst) == 0 && fst.status == st.status) {
          own = true;
          std::printf("Warning: the TLC-order re-run for the trace failed (%s); the trace below is a shortest "
                      "counterexample but may not be the one TLC prints, and the counts are at the end of the "
                      "level.\n", why.c_str());
        } else {
          tlcg_destroy(tctx);
          tctx = nullptr;
          std::printf("Warning: no trace: the re-run for it failed (%s).\n", why.c_str());
        }
      }
    }
    switch (tst.status) {
      case TLCG_VIOLATION:
        std::printf("Error: Invariant %s is violated%s.\n", cfg.invariants[(size_t)tst.invariant].c_str(),
                    tst.depth <= 1 && tst.event_gidx == ~0ull ? " by the initial state" : "");
        rc = 12;
        break;
      case TLCG_INVARIANT_ERROR:
        std::printf("Error: Evaluating invariant %s failed.\n", cfg.invariants[(size_t)tst.invariant].c_str());
        rc = 75;
        break;
      case TLCG_DEADLOCK:
        std::printf("Error: Deadlock reached.\n");
        rc = 11;
        break;
      default:
        std::printf("Error: Evaluating the next-state relation failed in action %s.\n",
                    tst.action >= 0 ? kActionName[tst.action] : "?");
        rc = 75;
        break;
    }
    if (o.trace && (tctx || use_node_trace)) {
      const int words = state_words;  // 1, or 2 for a > 63-bit layout
      std::vector<uint64_t> own_states;
      std::vector<int32_t> own_acts;
      if (!use_node_trace) {
        own_states.resize((size_t)words << 16);
        own_acts.resize(1 << 16);
      }
      std::vector<uint64_t>& states = use_node_trace ? node_states : own_states;
      std::vector<int32_t>& acts = use_node_trace ? node_acts : own_acts;
      int32_t n = use_node_trace ? std::min<int32_t>(node_tlen, (int32_t)acts.size()) : 0;
      if (use_node_trace || tlcg_trace_words(tctx, states.data(), acts.data(), (int32_t)acts.size(), &n) == 0) {
        std::printf("Error: The behavior up to this point is:\n");
        std::vector<char> buf(1 << 16);
        for (int i = 0; i < n; ++i) {
          if (acts[(size_t)i] < 0) std::printf("State %d: <Initial predicate>\n", i + 1);
          else std::printf("State %d: <%s>\n", i + 1, action_location(mod, acts[(size_t)i]).c_str());
          tlcg_decode_words(&model, &states[(size_t)i * words], buf.data(), (int32_t)buf.size());
          std::printf("%s\n\n", buf.data());
        }
      } else {
        std::printf("Error: %s\n", tlcg_last_error(tctx));
      }
    }
    // TLC stops mid-level: its counts at that moment (else the end of the level)
    uint64_t sg = 0, sd = 0, sq = 0;
    if (tctx && tlcg_tlc_stop_stats(tctx, &sg, &sd, &sq) == 0) {
      st.generated = sg;
      st.distinct = sd;
      stop_left = sq;
    } else if (tctx) {
      std::printf("Warning: TLC's counts at its stop could not be worked out (%s); the counts below are at the end "
                  "of the level.\n", tlcg_last_error(tctx));
    }
    if (own) tlcg_destroy(tctx);
  }
  std::printf("%llu states generated, %llu distinct states found, %llu states left on queue.\n",
              (unsigned long long)st.generated, (unsigned long long)st.distinct,
              (unsigned long long)(st.status == TLCG_DONE ? 0 : stop_left != ~0ull ? stop_left : st.frontier));
  std::printf("The depth of the complete state graph search is %d.\n", st.depth);
  // TLC's outdegree line (complete searches; needs TLC's first-discoverer parents)
  std::vector<uint64_t> od(4100);
  int32_t nod = 0;
  if (ctx && st.status == TLCG_DONE && tlcg_outdegree(ctx, od.data(), (int32_t)od.size(), &nod) == 0 && nod > 0) {
    // BucketStatistics: mean rounded; the 95th percentile is the first bucket
    // whose cumulative count reaches 0.95 of the observations
    uint64_t total = 0, weighted = 0, cum = 0;
    int mn = -1, p95 = 0;
    for (int k = 0; k < nod; ++k) {
      total += od[(size_t)k];
      weighted += (uint64_t)k * od[(size_t)k];
      if (mn < 0 && od[(size_t)k]) mn = k;
    }
    for (int k = 0; k < nod; ++k) {
      cum += od[(size_t)k];
      if ((double)cum >= 0.95 * (double)total) { p95 = k; break; }
    }
    std::printf("The average outdegree of the complete state graph is %lld (minimum is %d, the maximum %d and the 95th percentile is %d).\n",
                (long long)std::llround((double)weighted / (double)total), mn, nod - 1, p95);
  }
  double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  std::printf("Finished in %s at (%s)\n", duration_str(secs).c_str(), now_str().c_str());
  if (o.json) {
    std::printf("{\"status\": %d, \"generated\": %llu, \"distinct\": %llu, \"depth\": %d, \"kernel_ms\": %.3f, \"seconds\": %.4f}\n",
                st.status, (unsigned long long)st.generated, (unsigned long long)st.distinct, st.depth, st.kernel_ms,
                secs);
  }
  tlcg_destroy(ctx);
  return rc;
}
