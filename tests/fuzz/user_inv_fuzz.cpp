// Host-only fuzz harness for the user-invariant compiler (user_inv.cpp) and
// the model builder (host_model.cpp), built with -fsanitize=address,undefined
// by tests/test_user_inv_fuzz.py.  No GPU, no HIP runtime: the compiler, its
// interpreter (user_inv.h eval_user_v) and its device-code generator
// (user_device_source) are plain C++.
//
//   user_inv_fuzz CORPUS MUTANTS SEED
//
// CORPUS: entries "@@CASE <invariant name>" followed by a tlcg_model.user_defs
// text (the "@@DEF" headers and bodies of tlcgpu.Model.user_defs_text()).
// Every entry is compiled as written and as MUTANTS deterministic mutations
// (character drops, TLA+ token insertions, span duplications, truncations).
// A compile must end in a program or a message, never a crash or undefined
// behaviour; a program is generated as device code and evaluated by the
// interpreter on every reachable state of a small model, each result one of
// TRUE / FALSE / error.  Prints one summary line; exit 0 unless a check fails
// (the sanitizers abort on their own findings).
#include <cstdint>
#include <cstdio>
#include <fstream>
#include <sstream>
#include <string>
#include <unordered_set>
#include <vector>

#include "component_code.h"
#include "host_model.h"

namespace {

struct Entry {
  std::string name, text;
};

std::vector<Entry> read_corpus(const char* path) {
  std::ifstream f(path);
  std::vector<Entry> out;
  std::string line;
  while (std::getline(f, line)) {
    if (line.compare(0, 7, "@@CASE ") == 0) {
      out.push_back(Entry{line.substr(7), ""});
      continue;
    }
    if (!out.empty()) out.back().text += line + "\n";
  }
  return out;
}

struct Rng {
  uint64_t x;
  uint64_t next() {
    x ^= x << 13;
    x ^= x >> 7;
    x ^= x << 17;
    return x;
  }
  size_t below(size_t n) { return n ? (size_t)(next() % n) : 0; }
};

const char* const kTokens[] = {
    "\\A ", "\\E ", "(", ")", "[", "]", "{", "}", "..", " # ", " => ", "/\\ ", "\\/ ", "1", "0", "-1",
    "2147483647", "Len(", "messages", "compactedLedgers", "phaseOneResult", ".latestForKey", ".readPosition",
    "cursor", ".id", ".key", ".value", "CHOOSE x \\in ", "IF ", " THEN ", " ELSE ", "LET ", " IN ", ",", ":",
    " \\in ", " - ", " * ", " \\div ", " % ", " + ", " = ", " < ", " <= ", "~", "Nil", "DOMAIN ", "Head(",
    "Cardinality(", "KeySpace", "ValueSpace", "\n", "  ", "@@DEF X\n", "CASE ", " [] ", " -> ", "OTHER",
    "[i \\in 1..3 |-> i]", "<<1, 2>>", "TRUE", "FALSE", "x", "i", "\\cup ", "\\cap ", "SUBSET ", "\"s\""};

std::string mutate(const std::string& s, Rng& r) {
  std::string t = s;
  const int edits = 1 + (int)r.below(4);
  for (int e = 0; e < edits; ++e) {
    const size_t at = r.below(t.size() + 1);
    switch (r.below(5)) {
      case 0:  // drop a character
        if (!t.empty()) t.erase(r.below(t.size()), 1);
        break;
      case 1:  // insert a token
        t.insert(at, kTokens[r.below(sizeof kTokens / sizeof kTokens[0])]);
        break;
      case 2: {  // duplicate a span
        const size_t a = r.below(t.size() + 1), n = r.below(16);
        t.insert(at, t.substr(a, n));
        break;
      }
      case 3:  // truncate
        t.resize(at);
        break;
      default:  // replace a character with a printable one
        if (!t.empty()) t[r.below(t.size())] = (char)(32 + r.below(95));
        break;
    }
  }
  return t;
}

tlcg_model small_model() {
  tlcg_model m{};
  m.msg_sent_limit = 2;
  m.compaction_times_limit = 2;
  m.consume_times_limit = 0;
  m.max_crash_times = 1;
  m.retain_null_key = 1;
  m.check_deadlock = 1;
  m.n_keys = 2;
  m.keys[0] = 1;
  m.keys[1] = 2;
  m.n_values = 2;
  m.values[0] = 1;
  m.values[1] = 2;
  return m;
}

// every reachable state of the small model (words only: it fits 63 bits)
std::vector<uint64_t> reachable(const tlcg::HostModel& hm) {
  std::vector<uint64_t> all;
  std::unordered_set<uint64_t> seen;
  for (uint64_t i = 0; i < hm.n_init; ++i) {
    const uint64_t s = tlcg::init_state<uint64_t>(hm.L, i);
    if (seen.insert(s).second) all.push_back(s);
  }
  std::vector<uint64_t> out(256);
  for (size_t k = 0; k < all.size(); ++k) {
    const int n = tlcg::host_successors<uint64_t>(hm.L, all[k], out.data(), nullptr, (int)out.size());
    for (int j = 0; j < n; ++j)
      if (seen.insert(out[(size_t)j]).second) all.push_back(out[(size_t)j]);
  }
  return all;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 4) {
    std::fprintf(stderr, "usage: %s CORPUS MUTANTS SEED\n", argv[0]);
    return 2;
  }
  // the generated code's unrolled U_NTH (model.h ui_nth_n) against the
  // interpreter's scan (ui_nth), exhaustively over N <= 10 and every mask
  for (int n = 0; n <= 10; ++n) {
    struct {
      int N;
    } lay{n};
    for (uint64_t m = 0; m < (1ull << (n + 1)); ++m)  // (one bit past N: the fallback)
      for (long long j = -1; j <= n + 2; ++j)
        if (tlcg::ui_nth_n(lay, m, j) != tlcg::ui_nth(m, j)) {
          std::fprintf(stderr, "ui_nth_n differs: N %d mask %llx j %lld\n", n, (unsigned long long)m, j);
          return 1;
        }
  }
  const std::vector<Entry> corpus = read_corpus(argv[1]);
  const int mutants = std::atoi(argv[2]);
  Rng rng{std::strtoull(argv[3], nullptr, 10) | 1};
  tlcg::HostModel base;
  std::string err;
  tlcg_model m0 = small_model();
  if (!tlcg::build_model(m0, &base, &err)) {
    std::fprintf(stderr, "the small model does not build: %s\n", err.c_str());
    return 1;
  }
  const std::vector<uint64_t> states = reachable(base);
  long compiled = 0, refused = 0, evals = 0, trues = 0, falses = 0, errors = 0, unmutated_ok = 0;
  long tab_checks = 0, tab_wide = 0, static_checks = 0, static_wide = 0;
  for (const Entry& e : corpus) {
    for (int k = 0; k <= mutants; ++k) {
      const std::string text = k == 0 ? e.text : mutate(e.text, rng);
      const std::vector<std::string> names = tlcg::user_def_names(text.c_str());
      int idx = 0;
      for (size_t i = 0; i < names.size(); ++i)
        if (names[i] == e.name) idx = (int)i;
      tlcg_model m = small_model();
      m.n_invariants = 1;
      m.invariants[0] = TLCG_INV_USER + idx;
      m.user_defs = text.c_str();
      tlcg::HostModel hm;
      std::string msg;
      if (!tlcg::build_model(m, &hm, &msg)) {
        if (msg.empty()) {
          std::fprintf(stderr, "a refused compile without a message (case %s, mutant %d)\n", e.name.c_str(), k);
          return 1;
        }
        ++refused;
        continue;
      }
      ++compiled;
      if (k == 0) ++unmutated_ok;
      if (!hm.user) continue;  // (no user invariant named: nothing to evaluate)
      const std::string dev = tlcg::user_device_source(*hm.user, hm.L);
      if (dev.find("tlcg_user_eval") == std::string::npos) {
        std::fprintf(stderr, "device source without tlcg_user_eval (case %s)\n", e.name.c_str());
        return 1;
      }
      // the per-component outcome tables (component_code.h code_consts_user):
      // the program on a code equals its value on the pattern of the code
      // bits its fields take, unless that evaluation read past them (wide)
      const uint32_t fm = tlcg::code_field_mask(hm.L, tlcg::user_fields(*hm.user, 0));
      const int mb = hm.L.msg_sh + hm.L.N * hm.L.mw;
      const tlcg::UserProg pruned = tlcg::user_prune_dead(*hm.user);
      const bool reads_msgs = (tlcg::user_const_reads(*hm.user, 0) & 2u) != 0;
      for (uint64_t s : states) {
        const tlcg::CodeConsts kc = tlcg::code_consts(hm.L, tlcg::comp_msgs_init(hm.L, s));
        const tlcg::lkey lk = (tlcg::lkey)(s >> mb);
        const tlcg::ckey c = tlcg::code_encode(hm.L, lk);
        if ((s >> mb) != (uint64_t)lk || tlcg::code_decode(hm.L, kc, c) != lk) continue;
        const int direct = tlcg::eval_user_v(*hm.user, 0, tlcg::UVCode<uint64_t>{hm.L, kc, c});
        const tlcg::UVTab<uint64_t> v{{hm.L, kc, tlcg::code_pdep(tlcg::code_pext(c, fm), fm)}};
        const int tab = tlcg::eval_user_v(*hm.user, 0, v);
        ++tab_checks;
        if (v.wide) ++tab_wide;
        else if (tab != direct) {
          std::fprintf(stderr, "outcome table differs: case %s mutant %d state %llx: %d vs %d (fields %x)\n",
                       e.name.c_str(), k, (unsigned long long)s, tab, direct, tlcg::user_fields(*hm.user, 0));
          return 1;
        }
        // the host-made table of the state's class (Len, ledger content), for
        // a program that reads no `messages` (the static tables)
        if (!reads_msgs && kc.len <= (uint32_t)hm.L.N && tlcg::popcount32(fm) <= 5) {
          const uint64_t st = tlcg::user_static_table(pruned, hm.L, 0, fm, (int)kc.len, (uint32_t)(kc.ledbits >> 1));
          const int se = (int)((st >> (2 * tlcg::code_pext(c, fm))) & 3u);
          ++static_checks;
          if (se == 3) ++static_wide;
          else if (se != direct) {
            std::fprintf(stderr, "class table differs: case %s mutant %d state %llx: %d vs %d\n", e.name.c_str(), k,
                         (unsigned long long)s, se, direct);
            return 1;
          }
        }
      }
      for (uint64_t s : states) {
        const int r = tlcg::eval_user<uint64_t>(hm.L, *hm.user, 0, s);
        if (tlcg::eval_user<uint64_t>(hm.L, pruned, 0, s) != r) {
          std::fprintf(stderr, "the pruned program differs: case %s mutant %d state %llx\n", e.name.c_str(), k,
                       (unsigned long long)s);
          return 1;
        }
        ++evals;
        if (r == tlcg::EV_TRUE) ++trues;
        else if (r == tlcg::EV_FALSE) ++falses;
        else if (r == tlcg::EV_ERROR) ++errors;
        else {
          std::fprintf(stderr, "evaluation returned %d (case %s, mutant %d)\n", r, e.name.c_str(), k);
          return 1;
        }
      }
    }
  }
  std::printf("{\"entries\": %zu, \"unmutated_ok\": %ld, \"compiled\": %ld, \"refused\": %ld, \"states\": %zu, "
              "\"evals\": %ld, \"true\": %ld, \"false\": %ld, \"error\": %ld, \"table_checks\": %ld, "
              "\"table_wide\": %ld, \"static_checks\": %ld, \"static_wide\": %ld}\n",
              corpus.size(), unmutated_ok, compiled, refused, states.size(), evals, trues, falses, errors, tab_checks,
              tab_wide, static_checks, static_wide);
  return 0;
}
