// pulsar-tlaplus_amd/host/cfg.cpp -- TLC cfg parser, compaction.tla
// recognizer and constant binding (the ModelConfig / SpecProcessor /
// checkAssumptions roles of TLC for this spec).
#include "cfg.h"

#include <algorithm>
#include <cctype>
#include <cstdio>
#include <set>
#include <sstream>

namespace tlchost {

std::string Value::str() const {
  switch (kind) {
    case INT: return std::to_string(i);
    case STR: return "\"" + s + "\"";
    case BOOL: return i ? "TRUE" : "FALSE";
    case MODEL: return s;
    case SET: {
      std::string o = "{";
      for (size_t k = 0; k < set.size(); ++k) o += (k ? ", " : "") + set[k].str();
      return o + "}";
    }
  }
  return "?";
}

// ---------------- cfg tokenizer ----------------
namespace {

struct Tok {
  enum K { ID, NUM, STR, SYM, END } k = END;
  std::string t;
  int line = 0;
};

bool tokenize_cfg(const std::string& x, std::vector<Tok>* out, std::string* err) {
  size_t i = 0, n = x.size();
  int line = 1;
  while (i < n) {
    char c = x[i];
    if (c == '\n') { ++line; ++i; continue; }
    if (isspace((unsigned char)c)) { ++i; continue; }
    if (c == '\\' && i + 1 < n && x[i + 1] == '*') {  // line comment
      while (i < n && x[i] != '\n') ++i;
      continue;
    }
    if (c == '(' && i + 1 < n && x[i + 1] == '*') {  // nested block comment
      int depth = 0;
      while (i < n) {
        if (x[i] == '(' && i + 1 < n && x[i + 1] == '*') { ++depth; i += 2; continue; }
        if (x[i] == '*' && i + 1 < n && x[i + 1] == ')') { i += 2; if (--depth == 0) break; continue; }
        if (x[i] == '\n') ++line;
        ++i;
      }
      continue;
    }
    Tok t;
    t.line = line;
    if (isalpha((unsigned char)c) || c == '_') {
      size_t j = i;
      while (j < n && (isalnum((unsigned char)x[j]) || x[j] == '_')) ++j;
      t.k = Tok::ID; t.t = x.substr(i, j - i); i = j;
    } else if (isdigit((unsigned char)c) || (c == '-' && i + 1 < n && isdigit((unsigned char)x[i + 1]))) {
      size_t j = i + 1;
      while (j < n && isdigit((unsigned char)x[j])) ++j;
      t.k = Tok::NUM; t.t = x.substr(i, j - i); i = j;
    } else if (c == '"') {
      size_t j = i + 1;
      std::string s;
      while (j < n && x[j] != '"') {
        if (x[j] == '\\' && j + 1 < n) { s += x[j + 1]; j += 2; continue; }
        s += x[j++];
      }
      if (j >= n) { *err = "unterminated string in configuration file (line " + std::to_string(line) + ")"; return false; }
      t.k = Tok::STR; t.t = s; i = j + 1;
    } else if (c == '<' && i + 1 < n && x[i + 1] == '-') {
      t.k = Tok::SYM; t.t = "<-"; i += 2;
    } else if (c == '=' || c == ',' || c == '{' || c == '}' || c == '[' || c == ']') {
      t.k = Tok::SYM; t.t = std::string(1, c); ++i;
    } else {
      *err = std::string("unexpected character '") + c + "' in configuration file (line " + std::to_string(line) + ")";
      return false;
    }
    out->push_back(t);
  }
  Tok e;
  e.line = line;
  out->push_back(e);
  return true;
}

const std::set<std::string>& cfg_keywords() {
  static const std::set<std::string> k = {
      "CONSTANT", "CONSTANTS", "INIT", "NEXT", "SPECIFICATION", "INVARIANT", "INVARIANTS", "PROPERTY",
      "PROPERTIES", "CONSTRAINT", "CONSTRAINTS", "ACTION_CONSTRAINT", "ACTION_CONSTRAINTS", "SYMMETRY",
      "VIEW", "CHECK_DEADLOCK", "POSTCONDITION", "ALIAS"};
  return k;
}

struct CfgParser {
  std::vector<Tok> t;
  size_t p = 0;
  std::string* err;
  const Tok& cur() const { return t[p]; }
  bool is_kw() const { return cur().k == Tok::ID && cfg_keywords().count(cur().t); }
  bool fail(const std::string& m) {
    *err = "configuration file line " + std::to_string(cur().line) + ": " + m;
    return false;
  }
  bool value(Value* v) {
    const Tok& k = cur();
    if (k.k == Tok::NUM) { v->kind = Value::INT; v->i = std::stoll(k.t); ++p; return true; }
    if (k.k == Tok::STR) { v->kind = Value::STR; v->s = k.t; ++p; return true; }
    if (k.k == Tok::ID && !is_kw()) {
      if (k.t == "TRUE" || k.t == "FALSE") { v->kind = Value::BOOL; v->i = k.t == "TRUE"; ++p; return true; }
      v->kind = Value::MODEL; v->s = k.t; ++p; return true;
    }
    if (k.k == Tok::SYM && k.t == "{") {
      ++p;
      v->kind = Value::SET;
      if (cur().k == Tok::SYM && cur().t == "}") { ++p; return true; }
      for (;;) {
        Value e;
        if (!value(&e)) return false;
        v->set.push_back(e);
        if (cur().k == Tok::SYM && cur().t == ",") { ++p; continue; }
        if (cur().k == Tok::SYM && cur().t == "}") { ++p; return true; }
        return fail("expected ',' or '}' in a set");
      }
    }
    return fail("expected a value, found '" + k.t + "'");
  }
  bool names(std::vector<std::string>* out) {
    while (cur().k == Tok::ID && !is_kw()) {
      out->push_back(cur().t);
      ++p;
      if (cur().k == Tok::SYM && cur().t == ",") ++p;
    }
    return true;
  }
  bool run(Config* c) {
    while (cur().k != Tok::END) {
      if (!is_kw()) return fail("expected a keyword, found '" + cur().t + "'");
      std::string kw = cur().t;
      ++p;
      if (kw == "CONSTANT" || kw == "CONSTANTS") {
        while (cur().k == Tok::ID && !is_kw()) {
          std::string name = cur().t;
          ++p;
          if (cur().k == Tok::SYM && cur().t == "<-")
            return fail("definition override '" + name + " <- ...' is not supported by this checker");
          if (!(cur().k == Tok::SYM && cur().t == "=")) return fail("expected '=' after " + name);
          ++p;
          Value v;
          if (!value(&v)) return false;
          if (!c->constants.count(name)) c->order.push_back(name);
          c->constants[name] = v;
          if (cur().k == Tok::SYM && cur().t == ",") ++p;
        }
      } else if (kw == "INVARIANT" || kw == "INVARIANTS") {
        names(&c->invariants);
      } else if (kw == "PROPERTY" || kw == "PROPERTIES") {
        names(&c->properties);
      } else if (kw == "SPECIFICATION" || kw == "INIT" || kw == "NEXT") {
        if (cur().k != Tok::ID || is_kw()) return fail(kw + " needs a name");
        (kw == "SPECIFICATION" ? c->specification : kw == "INIT" ? c->init : c->next) = cur().t;
        ++p;
      } else if (kw == "CHECK_DEADLOCK") {
        if (cur().k != Tok::ID || (cur().t != "TRUE" && cur().t != "FALSE")) return fail("CHECK_DEADLOCK needs TRUE or FALSE");
        c->check_deadlock = cur().t == "TRUE";
        ++p;
      } else {
        return fail(kw + " is not supported by this checker");
      }
    }
    return true;
  }
};

// ---------------- module parsing ----------------

std::vector<std::string> split_lines(const std::string& s) {
  std::vector<std::string> v;
  std::string cur;
  for (char c : s) {
    if (c == '\n') { v.push_back(cur); cur.clear(); }
    else if (c != '\r') cur += c;
  }
  v.push_back(cur);
  return v;
}

// text of a line with `\*` comments removed (block comments handled by caller)
size_t code_end(const std::string& l) {
  size_t k = l.find("\\*");
  return k == std::string::npos ? l.size() : k;
}

std::string normalize(const std::string& s) {
  std::string o;
  bool sp = false;
  for (size_t i = 0; i < s.size(); ++i) {
    if (s[i] == '\\' && i + 1 < s.size() && s[i + 1] == '*') {  // to end of line
      while (i < s.size() && s[i] != '\n') ++i;
      sp = true;
      continue;
    }
    if (s[i] == '(' && i + 1 < s.size() && s[i + 1] == '*') {
      int d = 0;
      while (i < s.size()) {
        if (s[i] == '(' && i + 1 < s.size() && s[i + 1] == '*') { ++d; i += 2; continue; }
        if (s[i] == '*' && i + 1 < s.size() && s[i + 1] == ')') { i += 2; if (--d == 0) break; continue; }
        ++i;
      }
      --i;
      sp = true;
      continue;
    }
    if (isspace((unsigned char)s[i])) { sp = true; continue; }
    if (sp && !o.empty()) o += ' ';
    sp = false;
    o += s[i];
  }
  return o;
}

uint64_t fnv1a(const std::string& s) {
  uint64_t h = 1469598103934665603ull;
  for (unsigned char c : s) { h ^= c; h *= 1099511628211ull; }
  return h;
}

}  // namespace

bool parse_cfg(const std::string& text, Config* out, std::string* err) {
  CfgParser ps;
  ps.err = err;
  if (!tokenize_cfg(text, &ps.t, err)) return false;
  return ps.run(out);
}

bool parse_module(const std::string& text, Module* out, std::string* err) {
  std::vector<std::string> L = split_lines(text);
  Module m;
  // ---- MODULE name ----
  for (auto& l : L) {
    size_t k = l.find("MODULE");
    if (l.rfind("----", 0) == 0 && k != std::string::npos) {
      std::istringstream is(l.substr(k + 6));
      is >> m.name;
      break;
    }
  }
  if (m.name.empty()) { *err = "no ---- MODULE ---- header"; return false; }
  // Top-level items start at column 1.  A definition is "Name[(params)] ==".
  auto starts_item = [&](const std::string& l) {
    return !l.empty() && !isspace((unsigned char)l[0]);
  };
  const int nl = (int)L.size();
  for (int i = 0; i < nl; ++i) {
    const std::string& l = L[(size_t)i];
    if (!starts_item(l)) continue;
    size_t eq = l.find("==");
    bool is_assume = l.rfind("ASSUME", 0) == 0;
    if (eq == std::string::npos && !is_assume) continue;
    if (!is_assume && (l.rfind("----", 0) == 0 || l.rfind("====", 0) == 0 || l.rfind("\\*", 0) == 0)) continue;
    std::string head = is_assume ? "ASSUME" : l.substr(0, eq);
    std::string name;
    for (char c : head) { if (isalnum((unsigned char)c) || c == '_') name += c; else break; }
    if (name.empty()) continue;
    // body: from after "==" (or "ASSUME") to the last code char before the next item
    int j = i + 1;
    while (j < nl && !starts_item(L[(size_t)j])) ++j;
    size_t start_col = is_assume ? 6 : eq + 2;
    int l0 = i, c0 = -1;
    // first non-space code char of the body
    for (int a = i; a < j && c0 < 0; ++a) {
      const std::string& s = L[(size_t)a];
      size_t from = a == i ? start_col : 0, end = code_end(s);
      for (size_t b = from; b < end; ++b)
        if (!isspace((unsigned char)s[b])) { l0 = a; c0 = (int)b; break; }
    }
    int l1 = l0, c1 = c0;
    for (int a = j - 1; a >= l0; --a) {
      const std::string& s = L[(size_t)a];
      size_t end = code_end(s);
      size_t from = a == l0 ? (size_t)c0 : 0;
      int last = -1;
      for (size_t b = from; b < end; ++b)
        if (!isspace((unsigned char)s[b])) last = (int)b;
      if (last >= 0) { l1 = a; c1 = last; break; }
    }
    std::string body, text;
    for (int a = l0; a <= l1 && c0 >= 0; ++a) {
      const std::string& s = L[(size_t)a];
      size_t from = a == l0 ? (size_t)c0 : 0;
      size_t to = a == l1 ? (size_t)c1 + 1 : s.size();
      if (from < s.size()) body += s.substr(from, std::min(to, s.size()) - from);
      body += '\n';
      // the same lines with their columns (the first one's text before the body blanked)
      if (from < s.size()) text += std::string(from, ' ') + s.substr(from, std::min(to, s.size()) - from);
      text += '\n';
    }
    if (is_assume) {
      m.assume_l0 = l0 + 1; m.assume_c0 = c0 + 1; m.assume_l1 = l1 + 1; m.assume_c1 = c1 + 1;
      Def d;
      d.name = "ASSUME";
      d.line0 = l0 + 1; d.col0 = c0 + 1; d.line1 = l1 + 1; d.col1 = c1 + 1;
      d.norm = normalize(body);
      m.by_name[d.name] = m.defs.size();
      m.defs.push_back(d);
      continue;
    }
    Def d;
    d.name = name;
    d.line0 = l0 + 1; d.col0 = c0 + 1; d.line1 = l1 + 1; d.col1 = c1 + 1;
    d.norm = normalize(head + "==" + body);
    d.text = text;
    const size_t lp = head.find('('), rp = head.rfind(')');
    if (lp != std::string::npos && rp != std::string::npos && rp > lp) {
      std::string p;
      for (char ch : head.substr(lp + 1, rp - lp - 1) + ",") {
        if (ch == ',') {
          if (!p.empty()) d.params.push_back(p);
          p.clear();
        } else if (!isspace((unsigned char)ch)) {
          p += ch;
        }
      }
    }
    m.by_name[d.name] = m.defs.size();
    m.defs.push_back(d);
  }
  // declarations: CONSTANTS / VARIABLES blocks (names only)
  std::string decl;
  for (int i = 0; i < nl; ++i) {
    const std::string& l = L[(size_t)i];
    if (l.rfind("CONSTANT", 0) == 0 || l.rfind("VARIABLE", 0) == 0) {
      std::string block = l.substr(0, code_end(l)) + "\n";
      for (int j = i + 1; j < nl && !starts_item(L[(size_t)j]); ++j)
        block += L[(size_t)j].substr(0, code_end(L[(size_t)j])) + "\n";
      decl += normalize(block) + ";";
    }
  }
  Def dd;
  dd.name = "__DECLARATIONS__";
  dd.norm = decl;
  m.by_name[dd.name] = m.defs.size();
  m.defs.push_back(dd);
  *out = m;
  return true;
}

// Normalized-body fingerprints of the operators this build implements, taken
// from /root/reference/compaction.tla (FNV-1a over the text with comments
// removed and whitespace collapsed).  An edit to any of these (other than
// comments / layout) changes the model and is refused rather than mis-checked.
struct Known { const char* name; uint64_t h; int l0, c0, l1, c1; };  // fingerprint, body extent
static const Known kKnown[] = {
#include "known_defs.inc"
};

Module builtin_module() {
  Module m;
  m.name = "compaction";
  m.builtin = true;
  for (const Known& k : kKnown) {
    Def d;
    d.name = k.name;
    d.line0 = k.l0; d.col0 = k.c0; d.line1 = k.l1; d.col1 = k.c1;
    if (d.name == "ASSUME") {
      m.assume_l0 = k.l0; m.assume_c0 = k.c0; m.assume_l1 = k.l1; m.assume_c1 = k.c1;
    }
    m.by_name[d.name] = m.defs.size();
    m.defs.push_back(d);
  }
  return m;
}

bool recognize_compaction(const Module& m, std::string* err) {
  if (m.builtin) return true;  // the table itself
  std::vector<std::string> bad;
  if (m.name != "compaction") bad.push_back("MODULE name (" + m.name + ")");
  for (const Known& k : kKnown) {
    const Def* d = m.find(k.name);
    // the bug-reproducing / liveness definitions are only needed when referenced
    std::string n = k.name;
    bool optional = n == "CompactedLedgerLeak" || n == "DuplicateNullKeyMessage" || n == "Termination" ||
                    n == "TypeSafe" || n == "CompactionHorizonCorrectness";
    if (!d) { if (!optional) bad.push_back(n + " (missing)"); continue; }
    if (fnv1a(d->norm) != k.h && !optional) bad.push_back(n);
  }
  if (!bad.empty()) {
    std::string s = "this checker implements compaction.tla as published; these definitions differ:";
    for (auto& b : bad) s += " " + b;
    *err = s;
    return false;
  }
  return true;
}

// does the referenced invariant's body match the implemented one?
static bool invariant_matches(const Module& m, const std::string& name) {
  const Def* d = m.find(name);
  if (!d) return false;
  if (m.builtin && d->text.empty()) return true;  // (a definition added with -defs has its text)
  for (const Known& k : kKnown)
    if (name == k.name) return fnv1a(d->norm) == k.h;
  return false;
}

std::string user_defs_text(const Module& m, std::map<std::string, int>* index) {
  std::string out;
  int k = 0;
  for (const Def& d : m.defs) {
    if (d.name == "ASSUME" || d.name == "__DECLARATIONS__" || d.text.empty()) continue;
    out += "@@DEF " + d.name;
    for (const std::string& p : d.params) out += " " + p;
    out += " @" + std::to_string(d.line0) + "\n" + d.text;
    if (index) (*index)[d.name] = k;
    ++k;
  }
  return out;
}

bool bind_model(const Config& cfg, const Module& mod, bool deadlock_flag, tlcg_model* m, std::string* err,
                int* exit_code, int* fairness) {
  *m = tlcg_model();
  // [TLC-ext] EC.ExitStatus.ERROR_CONFIG_PARSE (151): the cfg does not bind the
  // module (150, ERROR_SPEC_PARSE, is the .tla's; 75 an evaluation error)
  *exit_code = 151;
  static const char* kParams[] = {"MessageSentLimit", "CompactionTimesLimit", "ModelConsumer", "ConsumeTimesLimit",
                                  "KeySpace", "ValueSpace", "RetainNullKey", "MaxCrashTimes", "ModelProducer"};
  static const char* kModelValues[] = {"Nil", "Compactor_In_PhaseOne", "Compactor_In_PhaseTwoWrite",
                                       "Compactor_In_PhaseTwoUpdateContext", "Compactor_In_PhaseTwoUpdateHorizon",
                                       "Compactor_In_PhaseTwoPersistCusror", "Compactor_In_PhaseTwoDeleteLedger"};
  std::set<std::string> declared(std::begin(kParams), std::end(kParams));
  for (auto* mv : kModelValues) declared.insert(mv);
  for (auto& kv : cfg.constants)
    if (!declared.count(kv.first)) {
      *err = "Error: The configuration file assigns a value to " + kv.first + ", which is not a CONSTANT of module " + mod.name + ".";
      return false;
    }
  for (auto* p : kParams)
    if (!cfg.constants.count(p)) {
      *err = std::string("Error: The constant parameter ") + p + " is not assigned a value by the configuration file.";
      return false;
    }
  for (auto* mv : kModelValues) {
    auto it = cfg.constants.find(mv);
    if (it == cfg.constants.end()) {
      *err = std::string("Error: The constant parameter ") + mv + " is not assigned a value by the configuration file.";
      return false;
    }
    if (it->second.kind != Value::MODEL) {
      *err = std::string("Error: this checker needs ") + mv + " bound to a model value (e.g. " + mv + " = " + mv + ").";
      return false;
    }
  }
  // distinct model values for the six phases and Nil (a TLC model value equals only itself)
  std::set<std::string> mvs;
  for (auto* mv : kModelValues) mvs.insert(cfg.constants.at(mv).s);
  if (mvs.size() != 7) {
    *err = "Error: this checker needs Nil and the six compactor states bound to distinct model values.";
    return false;
  }
  // ---- ASSUME, compaction.tla:25-35, conjuncts in order ----
  char loc[160];
  std::snprintf(loc, sizeof loc, "line %d, col %d to line %d, col %d of module %s", mod.assume_l0, mod.assume_c0,
                mod.assume_l1, mod.assume_c1, mod.name.c_str());
  auto assume_false = [&]() {
    *err = std::string("Error: Assumption ") + loc + " is false.";
    *exit_code = 10;  // [TLC-ext] EC.ExitStatus.VIOLATION_ASSUMPTION
    return false;
  };
  auto assume_error = [&](const std::string& msg) {
    *err = std::string("Error: Evaluating assumption ") + loc + " failed.\n" + msg;
    *exit_code = 75;  // [TLC-ext] evaluation error
    return false;
  };
  auto not_elem = [&](const Value& v, const std::string& set) {
    return "Attempted to check if the value:\n" + v.str() + "\nis an element of " + set + ".";
  };
  auto in_nat = [&](const char* n, int64_t* out) -> int {  // 1 true, 0 false, -1 error
    const Value& v = cfg.constants.at(n);
    if (v.kind == Value::INT) { *out = v.i; return v.i >= 0; }
    if (v.kind == Value::MODEL) return 0;
    assume_error(not_elem(v, "Nat"));
    return -1;
  };
  auto in_bool = [&](const char* n, bool* out) -> int {
    const Value& v = cfg.constants.at(n);
    if (v.kind == Value::BOOL) { *out = v.i != 0; return 1; }
    if (v.kind == Value::MODEL) return 0;
    assume_error("Attempted to check equality of a boolean with the value:\n" + v.str());
    return -1;
  };
  auto in_subset_nat = [&](const char* n, std::vector<int64_t>* out) -> int {
    const Value& v = cfg.constants.at(n);
    if (v.kind != Value::SET) {
      if (v.kind == Value::MODEL) return 0;
      assume_error(not_elem(v, "SUBSET Nat"));
      return -1;
    }
    // a TLC set is normalized (sorted) before it is enumerated: ints before
    // strings is irrelevant here, any non-int element errors
    std::vector<Value> el = v.set;
    std::stable_sort(el.begin(), el.end(), [](const Value& a, const Value& b) {
      if (a.kind != b.kind) return a.kind < b.kind;
      if (a.kind == Value::INT) return a.i < b.i;
      return a.s < b.s;
    });
    for (const Value& e : el) {
      if (e.kind == Value::INT) {
        if (e.i < 0) return 0;
        out->push_back(e.i);
      } else if (e.kind == Value::MODEL) {
        return 0;
      } else {
        assume_error(not_elem(e, "Nat"));
        return -1;
      }
    }
    std::sort(out->begin(), out->end());
    out->erase(std::unique(out->begin(), out->end()), out->end());
    return 1;
  };
  int64_t msl = 0, ctl = 0, ctl2 = 0, mct = 0;
  bool mc = false, rnk = false, mp = false;
  std::vector<int64_t> ks, vs;
  int r;
  if ((r = in_nat("MessageSentLimit", &msl)) <= 0) return r < 0 ? false : assume_false();
  if ((r = in_nat("CompactionTimesLimit", &ctl)) <= 0) return r < 0 ? false : assume_false();
  if ((r = in_bool("ModelConsumer", &mc)) <= 0) return r < 0 ? false : assume_false();
  if ((r = in_nat("ConsumeTimesLimit", &ctl2)) <= 0) return r < 0 ? false : assume_false();
  if ((r = in_subset_nat("KeySpace", &ks)) <= 0) return r < 0 ? false : assume_false();
  if (std::count(ks.begin(), ks.end(), 0)) return assume_false();
  if ((r = in_subset_nat("ValueSpace", &vs)) <= 0) return r < 0 ? false : assume_false();
  if (std::count(vs.begin(), vs.end(), 0)) return assume_false();
  if ((r = in_bool("RetainNullKey", &rnk)) <= 0) return r < 0 ? false : assume_false();
  if ((r = in_nat("MaxCrashTimes", &mct)) <= 0) return r < 0 ? false : assume_false();
  if ((r = in_bool("ModelProducer", &mp)) <= 0) return r < 0 ? false : assume_false();
  if (ks.size() > TLCG_MAX_SET || vs.size() > TLCG_MAX_SET) {
    *err = "Error: KeySpace/ValueSpace larger than this checker supports (63 elements).";
    return false;
  }
  // ---- behaviour spec ----
  if (fairness) *fairness = TLCG_FAIR_NONE;
  if (!cfg.specification.empty() && cfg.specification != "Spec") {
    // a fair specification the user adds to the module: Spec (compaction.tla:233)
    // conjoined with weak or strong fairness of Next; both ask that a
    // behavior never stutters forever where <<Next>>_vars is enabled, which is
    // the one property liveness checking needs from them (tlcg_check_termination)
    const Def* d = mod.find(cfg.specification);
    std::string body;
    if (d) {
      const size_t eq = d->norm.find("==");
      for (char ch : d->norm.substr(eq == std::string::npos ? 0 : eq + 2))
        if (!isspace((unsigned char)ch)) body += ch;
    }
    static const char* kFair[] = {"Spec/\\WF_vars(Next)", "Spec/\\SF_vars(Next)",
                                  "Init/\\[][Next]_vars/\\WF_vars(Next)", "Init/\\[][Next]_vars/\\SF_vars(Next)"};
    const bool fair = d && std::find(std::begin(kFair), std::end(kFair), body) != std::end(kFair);
    if (!fair) {
      *err = "Error: this checker supports SPECIFICATION Spec (compaction.tla:233), or a definition Spec /\\ "
             "WF_vars(Next) (or SF_vars(Next)), only.";
      return false;
    }
    if (fairness) *fairness = TLCG_FAIR_WF_NEXT;
  } else if (cfg.specification.empty() && (cfg.init != "Init" || cfg.next != "Next")) {
    *err = "Error: the configuration needs SPECIFICATION Spec or INIT Init / NEXT Next.";
    return false;
  }
  for (auto& name : cfg.properties) {
    if (!mod.find(name)) {
      *err = "Error: The property " + name + " specified in the configuration file is not defined in the specification.";
      return false;
    }
    if (name != "Termination" || !invariant_matches(mod, name)) {
      *err = "Error: temporal property " + name + " is not one this checker implements (Termination as published).";
      return false;
    }
  }
  m->msg_sent_limit = (int32_t)msl;
  m->compaction_times_limit = (int32_t)ctl;
  m->consume_times_limit = (int32_t)ctl2;
  m->max_crash_times = (int32_t)mct;
  m->model_consumer = mc;
  m->model_producer = mp;
  m->retain_null_key = rnk;
  bool dl = cfg.check_deadlock < 0 ? true : cfg.check_deadlock != 0;
  if (deadlock_flag) dl = false;  // TLC -deadlock: do not check for deadlock
  m->check_deadlock = dl;
  m->n_keys = (int32_t)ks.size();
  m->n_values = (int32_t)vs.size();
  for (size_t i = 0; i < ks.size(); ++i) m->keys[i] = ks[i];
  for (size_t i = 0; i < vs.size(); ++i) m->values[i] = vs[i];
  static const char* kInv[] = {"TypeSafe", "CompactedLedgerLeak", "CompactionHorizonCorrectness",
                               "DuplicateNullKeyMessage"};
  if (cfg.invariants.size() > TLCG_MAX_INV) {
    *err = "Error: too many invariants";
    return false;
  }
  m->n_invariants = 0;
  for (auto& name : cfg.invariants) {
    int id = -1;
    for (int q = 0; q < 4; ++q)
      if (name == kInv[q]) id = q;
    if (!mod.find(name)) {
      *err = "Error: The invariant " + name + " specified in the configuration file is not defined in the specification.";
      return false;
    }
    if (id < 0 || !invariant_matches(mod, name)) {
      // an invariant the user added (or edited): compiled from its text by
      // libtlcgpu (user_inv.cpp), which refuses what it cannot check exactly
      static std::string defs;  // (tlcg_model.user_defs points here)
      static std::map<std::string, int> index;
      if (!m->user_defs) {
        index.clear();
        defs = user_defs_text(mod, &index);
        m->user_defs = defs.c_str();
      }
      // a definition without body text (the built-in module's own Init, Next,
      // ...) is not in the index: refuse it rather than bind another one
      const auto it = index.find(name);
      if (it == index.end()) {
        *err = "Error: invariant " + name + " cannot be checked: its definition text is not available.";
        return false;  // (*exit_code is 151)
      }
      m->invariants[m->n_invariants++] = TLCG_INV_USER + it->second;
      continue;
    }
    m->invariants[m->n_invariants++] = id;
  }
  *exit_code = 0;
  return true;
}

}  // namespace tlchost
