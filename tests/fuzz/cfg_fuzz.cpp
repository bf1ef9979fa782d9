// Host-only fuzz harness for tlc-hip's front end (host/cfg.cpp: the TLC cfg
// parser, the module reader and its recognition, the constants binding),
// built with -fsanitize=address,undefined by tests/test_user_inv_fuzz.py.
//
//   cfg_fuzz CFG TLA MUTANTS SEED
//
// The cfg and the module are read as written and as MUTANTS deterministic
// mutations each (character drops, token insertions, span duplications,
// truncations); every parse and bind must end in a result or a message with
// an exit code, never a crash or undefined behaviour.  Prints one summary line.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <sstream>
#include <string>

#include "cfg.h"

namespace {

std::string slurp(const char* p) {
  std::ifstream f(p, std::ios::binary);
  std::ostringstream o;
  o << f.rdbuf();
  return o.str();
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

const char* const kTokens[] = {"CONSTANTS", "CONSTANT", "INVARIANT", "INVARIANTS", "PROPERTY", "SPECIFICATION",
                               "INIT", "NEXT", "CHECK_DEADLOCK", " = ", "{", "}", ",", "\"", "\\*", "(*", "*)",
                               "TRUE", "FALSE", "-1", "99999999999999999999", "\n", "  ", "==", "/\\", "\\/",
                               "----", "====", "MODULE", "EXTENDS", "VARIABLES", "ASSUME", "LET", "IN", "(", ")",
                               "[", "]", "\\A", "\\E", ":", "Nil", "KeySpace", "x"};

std::string mutate(const std::string& s, Rng& r) {
  std::string t = s;
  const int edits = 1 + (int)r.below(4);
  for (int e = 0; e < edits; ++e) {
    const size_t at = r.below(t.size() + 1);
    switch (r.below(5)) {
      case 0:
        if (!t.empty()) t.erase(r.below(t.size()), 1 + r.below(8));
        break;
      case 1:
        t.insert(at, kTokens[r.below(sizeof kTokens / sizeof kTokens[0])]);
        break;
      case 2: {
        const size_t a = r.below(t.size() + 1), n = r.below(64);
        t.insert(at, t.substr(a, n));
        break;
      }
      case 3:
        t.resize(at);
        break;
      default:
        if (!t.empty()) t[r.below(t.size())] = (char)(32 + r.below(95));
        break;
    }
  }
  return t;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 5) {
    std::fprintf(stderr, "usage: %s CFG TLA MUTANTS SEED\n", argv[0]);
    return 2;
  }
  const std::string cfg0 = slurp(argv[1]), tla0 = slurp(argv[2]);
  const int mutants = std::atoi(argv[3]);
  Rng rng{std::strtoull(argv[4], nullptr, 10) | 1};
  long cfg_ok = 0, cfg_bad = 0, mod_ok = 0, mod_bad = 0, recognized = 0, bound = 0, refused = 0;
  for (int k = 0; k <= mutants; ++k) {
    const bool mut_cfg = k > 0 && (k & 1), mut_tla = k > 0 && !(k & 1);
    const std::string cfg_text = mut_cfg ? mutate(cfg0, rng) : cfg0;
    const std::string tla_text = mut_tla ? mutate(tla0, rng) : tla0;
    tlchost::Config cfg;
    std::string err;
    if (!tlchost::parse_cfg(cfg_text, &cfg, &err)) {
      if (err.empty()) {
        std::fprintf(stderr, "cfg refused without a message (mutant %d)\n", k);
        return 1;
      }
      ++cfg_bad;
      continue;
    }
    ++cfg_ok;
    tlchost::Module mod;
    err.clear();
    if (!tlchost::parse_module(tla_text, &mod, &err)) {
      if (err.empty()) {
        std::fprintf(stderr, "module refused without a message (mutant %d)\n", k);
        return 1;
      }
      ++mod_bad;
      mod = tlchost::builtin_module();
    } else {
      ++mod_ok;
    }
    err.clear();
    if (tlchost::recognize_compaction(mod, &err)) ++recognized;
    std::map<std::string, int> index;
    (void)tlchost::user_defs_text(mod, &index);
    tlcg_model m{};
    int code = 0, fair = 0;
    err.clear();
    if (tlchost::bind_model(cfg, mod, false, &m, &err, &code, &fair)) {
      ++bound;
    } else {
      if (err.empty() || code == 0) {
        std::fprintf(stderr, "bind refused without a message or exit code (mutant %d)\n", k);
        return 1;
      }
      ++refused;
    }
  }
  std::printf("{\"cfg_ok\": %ld, \"cfg_bad\": %ld, \"module_ok\": %ld, \"module_bad\": %ld, \"recognized\": %ld, "
              "\"bound\": %ld, \"refused\": %ld}\n",
              cfg_ok, cfg_bad, mod_ok, mod_bad, recognized, bound, refused);
  return 0;
}
