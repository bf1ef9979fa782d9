// scripts/tree_probe_sim.cpp -- host simulation of the component tree's
// closed-mode FPSet (tree_body.h) on one component: the code BFS in the
// kernel's order (per depth, lanes in position order; each insert call is
// one wave-wide probe loop whose trip count is the longest probe of its
// lanes), reporting the probe trips the kernel pays with a given slot hash.
//   g++ -O2 -std=c++17 -I../include -Icsrc -o /tmp/tps ../scripts/tree_probe_sim.cpp -Llib -ltlcgpu
//   /tmp/tps KEYS C [TT] [MULT...]
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "component_code.h"
#include "host_model.h"

using namespace tlcg;

int main(int argc, char** argv) {
  const int k = argc > 1 ? std::atoi(argv[1]) : 10;
  tlcg_model m{};
  m.msg_sent_limit = 3;
  m.compaction_times_limit = argc > 2 ? std::atoi(argv[2]) : 12;
  m.consume_times_limit = 2;
  m.max_crash_times = 1;
  m.retain_null_key = 1;
  m.check_deadlock = 1;
  m.n_keys = m.n_values = k;
  for (int i = 0; i < k; ++i) m.keys[i] = m.values[i] = i + 1;
  m.n_invariants = 2;
  m.invariants[0] = TLCG_INV_TYPESAFE;
  m.invariants[1] = TLCG_INV_HORIZON_CORRECTNESS;
  HostModel hm;
  std::string err;
  if (!build_model(m, &hm, &err)) return std::fprintf(stderr, "%s\n", err.c_str()), 1;
  const Layout& L = hm.L;
  const int TT = argc > 3 ? std::atoi(argv[3]) : 640;
  std::vector<uint32_t> mults;
  for (int i = 4; i < argc; ++i) mults.push_back((uint32_t)std::strtoul(argv[i], nullptr, 0));
  if (mults.empty()) mults.push_back(0x9E3779B1u);
  const u128 s0 = init_state<u128>(L, 0);
  const CompMsgs cm = comp_msgs_init(L, (u64)s0);
  const CodeConsts kc = code_consts(L, cm);
  for (uint32_t mult : mults) {
    std::vector<uint32_t> h(TT, 0), keys;
    long trips = 0, probes = 0, calls = 0, maxp = 0;
    auto slot = [&](uint32_t key) { return (unsigned)(((unsigned long long)(key * mult) * (unsigned)TT) >> 32); };
    // one insert call: every lane's candidate probed; the loop runs to the longest probe
    auto insert_call = [&](const std::vector<std::pair<bool, uint32_t>>& cands) {
      int longest = 0;
      std::vector<uint32_t> added;
      for (auto& [pred, key] : cands) {
        if (!pred) continue;
        unsigned s = slot(key);
        int p = 0;
        if (std::getenv("BUCKET")) {  // 4-slot buckets: one 16-B read shows a bucket; the first empty slot takes the key
          unsigned b = s / 4;
          const unsigned nb = (unsigned)TT / 4;
          for (; p < TT; ++p) {
            bool done = false;
            for (int q = 0; q < 4 && !done; ++q) {
              uint32_t& e = h[b * 4 + q];
              if (e == key + 1) done = true;
              else if (e == 0) { e = key + 1; added.push_back(key); done = true; }
            }
            if (done) break;
            b = b + 1 == nb ? 0 : b + 1;
          }
        } else {
        for (; p < TT; ++p) {
          if (h[s] == 0) { h[s] = key + 1; added.push_back(key); break; }
          if (h[s] == key + 1) break;
          s = s + 1 == (unsigned)TT ? 0 : s + 1;
        }
        }
        longest = std::max(longest, p + 1);
        probes += p + 1;
        maxp = std::max(maxp, (long)p + 1);
      }
      trips += longest;
      ++calls;
      for (uint32_t a : added) keys.push_back(a);
    };
    insert_call({{true, code_encode_w<u128>(L, s0)}});
    size_t f0 = 0;
    int depth = 0;
    while (f0 < keys.size()) {
      const size_t f1 = keys.size();
      for (size_t b = f0; b < f1; b += 16) {
        std::vector<std::pair<bool, uint32_t>> c1, c2;
        for (size_t i = b; i < b + 16 && i < f1; ++i) {
          ckey t = 0, t2 = 0;
          int act = 0;
          const int r = compactor_step_cb(L, kc, keys[i], &t, &act);
          c1.push_back({r == 1, t});
          c2.push_back({crash_step_c(L, keys[i], &t2) != 0, t2});
        }
        insert_call(c1);
        insert_call(c2);
      }
      f0 = f1;
      ++depth;
    }
    std::printf("{\"mult\": \"0x%08x\", \"TT\": %d, \"states\": %zu, \"depths\": %d, \"insert_calls\": %ld, "
                "\"loop_trips\": %ld, \"probes\": %ld, \"max_probe\": %ld}\n",
                mult, TT, keys.size(), depth, calls, trips, probes, maxp);
  }
  return 0;
}
