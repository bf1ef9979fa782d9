// pulsar-tlaplus_amd/host/cfg.h -- TLC model-config parsing and binding of
// the compaction spec's constants (TLC's tlc2.tool.impl.ModelConfig role).
#pragma once
#include <cstdint>
#include <map>
#include <string>
#include <vector>

#include "tlcgpu.h"

namespace tlchost {

// A constant value as a TLC cfg writes it.
struct Value {
  enum Kind { INT, STR, BOOL, SET, MODEL } kind = INT;
  int64_t i = 0;
  std::string s;           // STR text or MODEL name
  std::vector<Value> set;  // SET elements (as written)
  std::string str() const;  // TLC print form
};

struct Config {
  std::map<std::string, Value> constants;  // CONSTANT(S) Name = value
  std::vector<std::string> order;          // constants in file order
  std::vector<std::string> invariants;     // INVARIANT(S), file order
  std::vector<std::string> properties;     // PROPERTY/PROPERTIES
  std::string specification, init, next;
  int check_deadlock = -1;                 // CHECK_DEADLOCK TRUE/FALSE, -1 unset
};

// Parses the TLC cfg grammar subset: CONSTANT(S), SPECIFICATION, INIT, NEXT,
// INVARIANT(S), PROPERTY/PROPERTIES, CHECK_DEADLOCK; `\*` and nested `(* *)`
// comments; values are integers, strings, TRUE/FALSE, {sets}, model values.
bool parse_cfg(const std::string& text, Config* out, std::string* err);

// A top-level definition of the module: name, text extent, normalized body.
struct Def {
  std::string name;
  int line0 = 0, col0 = 0, line1 = 0, col1 = 0;  // 1-based, inclusive: the body
  std::string norm;                               // whitespace/comment-normalized body
  std::vector<std::string> params;                // operator parameters
  std::string text;                               // the body as written, columns kept (user invariants)
};

struct Module {
  std::string name;
  bool builtin = false;  // built from known_defs.inc (no .tla text): fingerprints + extents only
  std::vector<Def> defs;
  std::map<std::string, size_t> by_name;
  int assume_l0 = 0, assume_c0 = 0, assume_l1 = 0, assume_c1 = 0;
  const Def* find(const std::string& n) const {
    auto it = by_name.find(n);
    return it == by_name.end() ? nullptr : &defs[it->second];
  }
};

bool parse_module(const std::string& text, Module* out, std::string* err);

// The module this build implements, from its compiled-in table (definition
// names, body fingerprints and source extents of compaction.tla -- numbers,
// not text): what tlc-hip checks when no .tla is given.
Module builtin_module();

// Checks that the module is the compaction spec this build implements
// (operator bodies compared after normalization); lists differing ones.
bool recognize_compaction(const Module& m, std::string* err);

// The module's definitions in tlcg_model.user_defs form ("@@DEF name params
// @line" + the body with its columns), for invariants the user added or
// edited (BASELINE config 5); *index gets each definition's position.
std::string user_defs_text(const Module& m, std::map<std::string, int>* index);

// Binds cfg constants to the model (ASSUME of compaction.tla:25-35 included).
// An INVARIANTS name that is not one of the spec's four as published becomes
// a user invariant (tlcg_model.user_defs, which then points into static
// storage of this file: one model bound per process).
// On failure `err` carries TLC-style text and `exit_code` TLC's exit status.
// `fairness` (may be null) gets the SPECIFICATION's fairness: TLCG_FAIR_NONE
// for Spec, TLCG_FAIR_WF_NEXT for a module definition Spec /\ WF_vars(Next).
bool bind_model(const Config& cfg, const Module& mod, bool deadlock_flag, tlcg_model* m, std::string* err,
                int* exit_code, int* fairness = nullptr);

}  // namespace tlchost
