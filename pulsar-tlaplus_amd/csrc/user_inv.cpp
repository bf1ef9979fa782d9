// pulsar-tlaplus_amd/csrc/user_inv.cpp -- compiler of user invariants
// (user_inv.h): TLA+ definitions -> register program over the packed state.
//
// Input (tlcg_model.user_defs): definitions, each introduced by a header line
//   @@DEF <name> [<param> ...]
// followed by the definition's body text with its original columns (TLA+
// bulleted /\ and \/ lists are read by column, as SANY does).  tlc-hip passes
// every non-action definition of the module; the Python face passes the
// definitions given to Model(user_defs=...).
//
// The expression language is TLA+'s, on the values this spec's states hold
// (compaction.tla:57-70): integers, booleans, the model values Nil and the six
// phases (:38-44), message records [id, key, value] (:80-81), sequences of
// messages (`messages`, every compacted ledger), the ledger function
// `compactedLedgers` (1..CompactionTimesLimit -> sequence or Nil), the cursor
// record (:150), phaseOneResult with its latestForKey function (:97-98), and
// sets of these.  Supported: /\ \/ ~ => <=> (infix and bulleted), = # /= < >
// <= >= \in \notin, + - * \div %, .., \cup \cap \ (set difference), IF THEN
// ELSE, LET IN (operators with parameters too), \A \E CHOOSE over sets,
// {e1, ..}, {x \in S : P}, {e : x \in S}, [f |-> e, ..] records,
// [f : S, ..] record sets, [x \in S |-> e] functions, f[x], r.f, Len,
// Cardinality, DOMAIN, Head, Nat, Int, BOOLEAN, and every definition of the
// module (by substitution, as TLA+ operators are).  Anything else is refused
// with a message naming it; an invariant is never checked approximately.
//
// Static typing resolves composites at compile time; what is left is 64-bit
// integer work (user_inv.h).  TLC's evaluation order is kept where it decides
// between FALSE and an evaluation error: /\, \/, => and IF short-circuit left
// to right, quantifiers and CHOOSE evaluate their whole set before their body
// (TLC enumerates the set first), Len of a function constructor evaluates it.
#include "user_inv.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <set>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "component_code.h"
#include "host_model.h"

namespace tlcg {

namespace {

struct CompileError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

// ---------------------------------------------------------------- lexer
struct Tok {
  enum K { ID, NUM, STR, OP, END } k = END;
  std::string s;
  long long v = 0;
  int line = 0, col = 0;
};

std::vector<Tok> lex(const std::string& text, int line0) {
  std::vector<Tok> out;
  static const char* kMulti[] = {"<=>", "|->", "==", "/\\", "\\/", "=>", "/=", "<=", "=<", ">=", "..", "<<", ">>", "->",
                                 "[]"};
  int line = line0, col = 1;
  size_t i = 0;
  auto adv = [&](size_t n) {
    for (size_t k = 0; k < n && i < text.size(); ++k, ++i) {
      if (text[i] == '\n') {
        ++line;
        col = 1;
      } else {
        ++col;
      }
    }
  };
  while (i < text.size()) {
    const char ch = text[i];
    if (ch == ' ' || ch == '\t' || ch == '\r' || ch == '\n') {
      adv(1);
      continue;
    }
    if (ch == '\\' && i + 1 < text.size() && text[i + 1] == '*') {  // \* comment
      while (i < text.size() && text[i] != '\n') adv(1);
      continue;
    }
    if (ch == '(' && i + 1 < text.size() && text[i + 1] == '*') {  // (* nested *)
      int depth = 0;
      while (i < text.size()) {
        if (text.compare(i, 2, "(*") == 0) {
          ++depth;
          adv(2);
        } else if (text.compare(i, 2, "*)") == 0) {
          adv(2);
          if (--depth == 0) break;
        } else {
          adv(1);
        }
      }
      continue;
    }
    Tok t;
    t.line = line;
    t.col = col;
    if (std::isalpha((unsigned char)ch) || ch == '_') {
      size_t j = i;
      while (j < text.size() && (std::isalnum((unsigned char)text[j]) || text[j] == '_')) ++j;
      t.k = Tok::ID;
      t.s = text.substr(i, j - i);
      adv(j - i);
    } else if (std::isdigit((unsigned char)ch)) {
      size_t j = i;
      while (j < text.size() && std::isdigit((unsigned char)text[j])) ++j;
      t.k = Tok::NUM;
      t.s = text.substr(i, j - i);
      t.v = std::stoll(t.s);
      adv(j - i);
    } else if (ch == '"') {
      size_t j = i + 1;
      while (j < text.size() && text[j] != '"') ++j;
      t.k = Tok::STR;
      t.s = text.substr(i + 1, j - i - 1);
      adv(j + 1 - i);
    } else if (ch == '\\' && i + 1 < text.size() && std::isalpha((unsigned char)text[i + 1])) {
      size_t j = i + 1;
      while (j < text.size() && std::isalpha((unsigned char)text[j])) ++j;
      t.k = Tok::OP;
      t.s = text.substr(i, j - i);
      adv(j - i);
    } else {
      t.k = Tok::OP;
      bool found = false;
      for (const char* m : kMulti) {
        const size_t n = std::strlen(m);
        if (text.compare(i, n, m) == 0) {
          t.s = m;
          adv(n);
          found = true;
          break;
        }
      }
      if (!found) {
        t.s = std::string(1, ch);
        adv(1);
      }
    }
    out.push_back(t);
  }
  Tok e;
  e.k = Tok::END;
  e.line = line;
  e.col = 0;
  out.push_back(e);
  return out;
}

// ---------------------------------------------------------------- AST
struct Node;
typedef std::shared_ptr<Node> NodeP;
struct Node {
  enum K {
    NUM, BOOL, STR, ID, OPAPP, BIN, UN, IF, LET, QUANT, CHOOSE, SETENUM, SETFILTER, SETMAP, APP, FIELD, RECORD,
    RECSET, FCTOR, TUPLE, JUNCT, DOMAIN, CASE
  } k;
  std::string s;                     // name, operator, field, quantifier (\A / \E), junction (/\ or \/)
  long long v = 0;
  std::vector<NodeP> c;
  std::vector<std::string> names;    // bound variables / record fields / LET names
  std::vector<std::vector<std::string>> params;  // LET operator parameters
  int line = 0, col = 0;
};

NodeP mk(Node::K k, const Tok& at) {
  auto n = std::make_shared<Node>();
  n->k = k;
  n->line = at.line;
  n->col = at.col;
  return n;
}

std::string where(int line, int col) {
  return "line " + std::to_string(line) + ", col " + std::to_string(col);
}

// ---------------------------------------------------------------- parser
class Parser {
 public:
  explicit Parser(std::vector<Tok> t) : t_(std::move(t)) {}

  NodeP parse_all() {
    NodeP e = expr(0);
    if (peek().k != Tok::END) fail("unexpected '" + peek().s + "'");
    return e;
  }

 private:
  std::vector<Tok> t_;
  size_t p_ = 0;
  std::vector<int> fence_;  // columns of the enclosing bulleted lists: a token at or left of one ends the item

  [[noreturn]] void fail(const std::string& m) const {
    const Tok& t = t_[std::min(p_, t_.size() - 1)];
    throw CompileError(m + " at " + where(t.line, t.col));
  }
  const Tok& peek(size_t k = 0) const {
    static Tok end;
    const size_t q = p_ + k;
    if (q >= t_.size()) return t_.back();
    const Tok& t = t_[q];
    if (!fence_.empty() && t.k != Tok::END && t.col <= fence_.back() && k == 0 && fenced_) return end;
    return t;
  }
  bool fenced_ = true;
  bool is(const char* s) const { return peek().k == Tok::OP && peek().s == s; }
  bool is_id(const char* s) const { return peek().k == Tok::ID && peek().s == s; }
  Tok next() {
    if (peek().k == Tok::END) fail("unexpected end of the definition");
    return t_[p_++];
  }
  void expect(const char* s) {
    if (!(is(s) || is_id(s))) fail(std::string("expected '") + s + "'");
    ++p_;
  }
  std::string ident() {
    if (peek().k != Tok::ID) fail("expected an identifier");
    return t_[p_++].s;
  }

  // binary operators: precedence (TLA+ book, table of operators), left-assoc?
  static bool binop(const Tok& t, int* prec, bool* left, std::string* op) {
    if (t.k != Tok::OP && !(t.k == Tok::ID && false)) return false;
    std::string s = t.s;
    if (s == "\\land") s = "/\\";
    if (s == "\\lor") s = "\\/";
    if (s == "\\equiv") s = "<=>";
    if (s == "=<" || s == "\\leq") s = "<=";
    if (s == "\\geq") s = ">=";
    if (s == "/=") s = "#";
    if (s == "\\union") s = "\\cup";
    if (s == "\\intersect") s = "\\cap";
    struct P { const char* o; int p; bool l; };
    static const P tab[] = {{"=>", 1, false}, {"<=>", 2, false}, {"/\\", 3, true}, {"\\/", 3, true},
                            {"=", 5, false},  {"#", 5, false},   {"<", 5, false},  {">", 5, false},
                            {"<=", 5, false}, {">=", 5, false},  {"\\in", 5, false}, {"\\notin", 5, false},
                            {"\\subseteq", 5, false}, {"\\cup", 8, true}, {"\\cap", 8, true}, {"\\", 8, true},
                            {"..", 9, false}, {"+", 10, true}, {"-", 10, true}, {"*", 13, true},
                            {"\\div", 13, true}, {"%", 10, false}};
    for (const P& x : tab)
      if (s == x.o) {
        *prec = x.p;
        *left = x.l;
        *op = s;
        return true;
      }
    return false;
  }

  NodeP expr(int min_prec) {
    NodeP lhs = unary();
    for (;;) {
      int prec = 0;
      bool left = true;
      std::string op;
      const Tok& t = peek();
      if (!binop(t, &prec, &left, &op) || prec < min_prec) break;
      const Tok at = next();
      NodeP rhs = expr(left ? prec + 1 : prec + 1);
      NodeP b = mk(Node::BIN, at);
      b->s = op;
      b->c = {lhs, rhs};
      lhs = b;
      if (!left) {  // non-associative / right: a second one at the same level is an error in TLA+
        int p2 = 0;
        bool l2;
        std::string o2;
        if (binop(peek(), &p2, &l2, &o2) && p2 == prec && prec != 1) fail("ambiguous '" + o2 + "' (add parentheses)");
      }
    }
    return lhs;
  }

  NodeP unary() {
    const Tok& t = peek();
    if (t.k == Tok::OP && (t.s == "~" || t.s == "\\lnot" || t.s == "\\neg")) {
      const Tok at = next();
      NodeP n = mk(Node::UN, at);
      n->s = "~";
      n->c = {expr(4)};
      return n;
    }
    if (t.k == Tok::OP && t.s == "-") {
      const Tok at = next();
      NodeP n = mk(Node::UN, at);
      n->s = "-";
      n->c = {expr(12)};
      return n;
    }
    return postfix(primary());
  }

  NodeP postfix(NodeP e) {
    for (;;) {
      if (is("[")) {
        const Tok at = next();
        NodeP a = mk(Node::APP, at);
        NodeP arg = expr(0);
        if (is(",")) fail("functions of several arguments are not supported");
        expect("]");
        a->c = {e, arg};
        e = a;
      } else if (is(".") && peek(1).k == Tok::ID) {
        const Tok at = next();
        NodeP f = mk(Node::FIELD, at);
        f->s = ident();
        f->c = {e};
        e = f;
      } else if (is("'")) {
        fail("primed variables are not state predicates");
      } else {
        return e;
      }
    }
  }

  // a bulleted /\ or \/ list whose first bullet is the next token
  NodeP junction() {
    const Tok b = next();
    NodeP j = mk(Node::JUNCT, b);
    j->s = b.s == "\\land" ? "/\\" : b.s == "\\lor" ? "\\/" : b.s;
    for (;;) {
      fence_.push_back(b.col);
      NodeP item = expr(0);
      fence_.pop_back();
      j->c.push_back(item);
      // the next bullet of this list: same operator at exactly the list's column
      fenced_ = false;
      const Tok& n = peek();
      const bool more = n.k == Tok::OP && n.col == b.col && (n.s == b.s) &&
                        (fence_.empty() || n.col > fence_.back());
      fenced_ = true;
      if (!more) break;
      ++p_;
    }
    return j;
  }

  void bound(NodeP q, bool allow_tuple = false) {
    (void)allow_tuple;
    // x \in S, y \in T   or   x, y \in S
    std::vector<std::pair<std::vector<std::string>, NodeP>> groups;
    for (;;) {
      std::vector<std::string> vs = {ident()};
      while (is(",")) {
        ++p_;
        vs.push_back(ident());
      }
      expect("\\in");
      NodeP s = expr(6);
      groups.push_back({vs, s});
      if (!is(",")) break;
      ++p_;
    }
    for (auto& g : groups)
      for (auto& v : g.first) {
        q->names.push_back(v);
        q->c.push_back(g.second);
      }
  }

  NodeP primary() {
    const Tok& t = peek();
    if (t.k == Tok::END) fail("expression expected");
    if (t.k == Tok::NUM) {
      const Tok at = next();
      NodeP n = mk(Node::NUM, at);
      n->v = at.v;
      return n;
    }
    if (t.k == Tok::STR) {
      const Tok at = next();
      NodeP n = mk(Node::STR, at);
      n->s = at.s;
      return n;
    }
    if (t.k == Tok::OP && (t.s == "/\\" || t.s == "\\/" || t.s == "\\land" || t.s == "\\lor")) return junction();
    if (t.k == Tok::OP && (t.s == "[]" || (t.s == "<" && peek(1).k == Tok::OP && peek(1).s == ">")))
      fail("a temporal formula ([] or <>) is not a state predicate");
    if (t.k == Tok::OP && t.s == "(") {
      ++p_;
      fence_.push_back(-1);  // parentheses lift the bullet fence
      NodeP e = expr(0);
      fence_.pop_back();
      expect(")");
      return e;
    }
    if (t.k == Tok::OP && (t.s == "\\A" || t.s == "\\E" || t.s == "\\forall" || t.s == "\\exists")) {
      const Tok at = next();
      NodeP q = mk(Node::QUANT, at);
      q->s = (at.s == "\\A" || at.s == "\\forall") ? "A" : "E";
      bound(q);
      expect(":");
      q->c.push_back(expr(0));
      return q;
    }
    if (t.k == Tok::ID) {
      if (t.s == "TRUE" || t.s == "FALSE") {
        const Tok at = next();
        NodeP n = mk(Node::BOOL, at);
        n->v = at.s == "TRUE";
        return n;
      }
      if (t.s == "IF") {
        const Tok at = next();
        NodeP n = mk(Node::IF, at);
        NodeP c = expr(0);
        expect("THEN");
        NodeP a = expr(0);
        expect("ELSE");
        NodeP b = expr(0);
        n->c = {c, a, b};
        return n;
      }
      if (t.s == "CASE") {
        const Tok at = next();
        NodeP n = mk(Node::CASE, at);
        for (;;) {
          if (is_id("OTHER")) {
            ++p_;
            expect("->");
            n->c.push_back(nullptr);
            n->c.push_back(expr(0));
            break;
          }
          n->c.push_back(expr(0));
          expect("->");
          n->c.push_back(expr(0));
          if (!is("[]")) break;
          ++p_;
        }
        return n;
      }
      if (t.s == "LET") {
        const Tok at = next();
        NodeP n = mk(Node::LET, at);
        while (!is_id("IN")) {
          n->names.push_back(ident());
          std::vector<std::string> ps;
          if (is("(")) {
            ++p_;
            ps.push_back(ident());
            while (is(",")) {
              ++p_;
              ps.push_back(ident());
            }
            expect(")");
          }
          n->params.push_back(ps);
          expect("==");
          fence_.push_back(-1);
          n->c.push_back(expr(0));
          fence_.pop_back();
        }
        expect("IN");
        n->c.push_back(expr(0));
        return n;
      }
      if (t.s == "CHOOSE") {
        const Tok at = next();
        NodeP n = mk(Node::CHOOSE, at);
        n->names.push_back(ident());
        expect("\\in");
        n->c.push_back(expr(6));
        expect(":");
        n->c.push_back(expr(0));
        return n;
      }
      if (t.s == "DOMAIN") {
        const Tok at = next();
        NodeP n = mk(Node::DOMAIN, at);
        n->c = {postfix(primary())};
        return n;
      }
      if (t.s == "LAMBDA" || t.s == "EXCEPT" || t.s == "SUBSET" || t.s == "UNION" || t.s == "ENABLED" ||
          t.s == "UNCHANGED")
        fail("'" + t.s + "' is not supported in an invariant");
      const Tok at = next();
      if (is("(")) {  // operator application Name(args)
        ++p_;
        NodeP n = mk(Node::OPAPP, at);
        n->s = at.s;
        fence_.push_back(-1);
        n->c.push_back(expr(0));
        while (is(",")) {
          ++p_;
          n->c.push_back(expr(0));
        }
        fence_.pop_back();
        expect(")");
        return n;
      }
      NodeP n = mk(Node::ID, at);
      n->s = at.s;
      return n;
    }
    if (t.k == Tok::OP && t.s == "{") {
      const Tok at = next();
      fence_.push_back(-1);
      NodeP r;
      if (is("}")) {
        r = mk(Node::SETENUM, at);
      } else if (peek().k == Tok::ID && peek(1).k == Tok::OP && peek(1).s == "\\in" && scan_filter()) {
        r = mk(Node::SETFILTER, at);  // {x \in S : P}
        r->names.push_back(ident());
        expect("\\in");
        r->c.push_back(expr(6));
        expect(":");
        r->c.push_back(expr(0));
      } else {
        NodeP first = expr(0);
        if (is(":")) {  // {e : x \in S}
          ++p_;
          r = mk(Node::SETMAP, at);
          r->c.push_back(first);
          bound(r);
        } else {
          r = mk(Node::SETENUM, at);
          r->c.push_back(first);
          while (is(",")) {
            ++p_;
            r->c.push_back(expr(0));
          }
        }
      }
      fence_.pop_back();
      expect("}");
      return r;
    }
    if (t.k == Tok::OP && t.s == "<<") {
      const Tok at = next();
      NodeP n = mk(Node::TUPLE, at);
      fence_.push_back(-1);
      if (!is(">>")) {
        n->c.push_back(expr(0));
        while (is(",")) {
          ++p_;
          n->c.push_back(expr(0));
        }
      }
      fence_.pop_back();
      expect(">>");
      return n;
    }
    if (t.k == Tok::OP && t.s == "[") {
      const Tok at = next();
      fence_.push_back(-1);
      NodeP n;
      // [x \in S |-> e], [f |-> e, ..], [f : S, ..]
      if (peek().k == Tok::ID && peek(1).k == Tok::OP && peek(1).s == "\\in") {
        n = mk(Node::FCTOR, at);
        n->names.push_back(ident());
        expect("\\in");
        n->c.push_back(expr(6));
        if (is(",")) fail("functions of several arguments are not supported");
        expect("|->");
        n->c.push_back(expr(0));
      } else if (peek().k == Tok::ID && peek(1).k == Tok::OP && peek(1).s == "|->") {
        n = mk(Node::RECORD, at);
        for (;;) {
          n->names.push_back(ident());
          expect("|->");
          n->c.push_back(expr(0));
          if (!is(",")) break;
          ++p_;
        }
      } else if (peek().k == Tok::ID && peek(1).k == Tok::OP && peek(1).s == ":") {
        n = mk(Node::RECSET, at);
        for (;;) {
          n->names.push_back(ident());
          expect(":");
          n->c.push_back(expr(0));
          if (!is(",")) break;
          ++p_;
        }
      } else {
        fail("unsupported bracket expression ([S -> T], EXCEPT)");
      }
      fence_.pop_back();
      expect("]");
      return n;
    }
    fail("unexpected '" + t.s + "'");
  }

  // after "{ x \in": is this {x \in S : P} (a ':' at nesting depth 0 before '}')?
  bool scan_filter() const {
    int depth = 0;
    for (size_t q = p_ + 2; q < t_.size(); ++q) {
      const Tok& t = t_[q];
      if (t.k == Tok::END) return false;
      if (t.k != Tok::OP) continue;
      if (t.s == "(" || t.s == "[" || t.s == "{" || t.s == "<<") ++depth;
      else if (t.s == ")" || t.s == "]" || t.s == ">>") --depth;
      else if (t.s == "}") {
        if (depth == 0) return false;
        --depth;
      } else if (t.s == ":" && depth == 0) {
        return true;
      } else if (t.s == "," && depth == 0) {
        return false;
      }
    }
    return false;
  }
};

// ---------------------------------------------------------------- types / values
enum TK { T_INT, T_BOOL, T_MV, T_MSG, T_SEQ, T_LEDGERS, T_CUR, T_P1R, T_LFK, T_SET, T_FUNC, T_REC };

const char* tk_name(TK t) {
  static const char* n[] = {"integer", "boolean", "model value", "message record", "sequence of messages",
                            "compactedLedgers", "cursor record", "phaseOneResult record", "latestForKey function",
                            "set", "function", "record"};
  return n[t];
}

struct Def {
  std::string name;
  std::vector<std::string> params;
  std::string text;
  int line0 = 0;
  NodeP body;       // parsed on first use
  std::string err;  // parse error
  bool parsed = false;
};

struct Env;
typedef std::shared_ptr<Env> EnvP;

// a value in registers (or, for sets and functions, an unevaluated expression)
struct Val {
  TK t = T_INT;
  int r[4] = {-1, -1, -1, -1};  // INT/BOOL/MV: r0; MSG: id key value; SEQ: mask; CUR: h c; P1R/LFK: readPosition
  int nil = -1;                 // composite that may be Nil: register holding 1 when it is; -1 = never Nil
  NodeP node;                   // T_SET / T_FUNC: the expression, and its environment
  EnvP env;
  bool nil_literal = false;     // T_MV: the constant Nil
};

struct Bind {
  bool by_name = true;  // an unevaluated expression (LET definition, operator argument)
  bool own_env = false; // a LET definition: its environment is the one that holds it (not held
                        // here, which would be a reference cycle)
  NodeP node;
  EnvP env;
  std::vector<std::string> params;
  Val v;                // by_name = false: a value in registers (bound variable)
};

struct Env : std::enable_shared_from_this<Env> {
  std::map<std::string, Bind> m;
  EnvP up;
  // the binding of n, and (owner) the environment that holds it
  const Bind* find(const std::string& n, const Env** owner = nullptr) const {
    for (const Env* e = this; e; e = e->up.get()) {
      auto it = e->m.find(n);
      if (it != e->m.end()) {
        if (owner) *owner = e;
        return &it->second;
      }
    }
    return nullptr;
  }
};

class Compiler {
 public:
  Compiler(const HostModel& hm, UserProg* P) : L_(hm.L), P_(P) {}

  std::map<std::string, Def> defs;

  // compiles definition `name` as user invariant k
  void compile(int k, const std::string& name) {
    auto it = defs.find(name);
    if (it == defs.end()) throw CompileError("invariant " + name + " is not defined");
    if (!it->second.params.empty()) throw CompileError("invariant " + name + " takes arguments");
    P_->entry[k] = pc();
    nreg_ = 0;
    EnvP env = std::make_shared<Env>();
    const Val v = lower(body_of(it->second), env);
    if (v.t != T_BOOL) throw CompileError("invariant " + name + " is a " + tk_name(v.t) + ", not a boolean");
    emit(U_RET, v.r[0]);
  }

 private:
  const Layout& L_;
  UserProg* P_;
  int nreg_ = 0;
  int depth_ = 0;
  int dry_ = 0;  // > 0: type probing (code is discarded)

  int pc() const { return P_->n_ins; }
  int emit(int op, int a = 0, int b = 0, int c = 0, int imm = 0) {
    if (P_->n_ins >= UI_MAXINS) throw CompileError("the invariants need more than " + std::to_string(UI_MAXINS) +
                                                   " instructions");
    UInsn& in = P_->ins[P_->n_ins];
    in.op = (uint8_t)op;
    in.a = (uint8_t)a;
    in.b = (uint8_t)b;
    in.c = (uint8_t)c;
    in.imm = imm;
    return P_->n_ins++;
  }
  void patch(int at, int target) { P_->ins[at].imm = target; }
  int R() {
    if (nreg_ >= UI_MAXREG) throw CompileError("the invariant needs more than " + std::to_string(UI_MAXREG) +
                                               " registers");
    return nreg_++;
  }
  int ldi(long long v) {
    const int r = R();
    emit(U_LDI, r, 0, 0, (int32_t)v);
    return r;
  }
  [[noreturn]] void fail(const NodeP& n, const std::string& m) {
    throw CompileError(m + (n ? " at " + where(n->line, n->col) : std::string()));
  }

  NodeP body_of(Def& d) {
    if (!d.parsed) {
      d.parsed = true;
      try {
        Parser p(lex(d.text, d.line0));
        d.body = p.parse_all();
      } catch (const CompileError& e) {
        d.err = e.what();
      }
    }
    if (!d.body) throw CompileError("definition " + d.name + ": " + d.err);
    return d.body;
  }

  // the type of an expression, by compiling it and throwing the code away
  Val probe(const NodeP& n, const EnvP& env) {
    const int n_ins = P_->n_ins, nr = nreg_;
    ++dry_;
    Val v;
    try {
      v = lower(n, env);
    } catch (...) {
      --dry_;
      P_->n_ins = n_ins;
      nreg_ = nr;
      throw;
    }
    --dry_;
    P_->n_ins = n_ins;
    nreg_ = nr;
    return v;
  }

  // ---- values of the state and the constants
  Val var_or_const(const NodeP& n) {
    const std::string& s = n->s;
    Val v;
    auto reg1 = [&](int op) {
      v.r[0] = R();
      emit(op, v.r[0]);
    };
    if (s == "messages") {  // the whole sequence: positions 1..Len
      v.t = T_SEQ;
      const int len = R();
      emit(U_LEN, len);
      v.r[0] = R();
      emit(U_MASK, v.r[0], len);
      return v;
    }
    if (s == "compactedLedgers") {
      v.t = T_LEDGERS;
      return v;
    }
    if (s == "cursor") {
      v.t = T_CUR;
      const int p = R();
      emit(U_CURP, p);
      v.nil = R();
      emit(U_NOT, v.nil, p);
      v.r[0] = R();
      emit(U_CURH, v.r[0]);
      v.r[1] = R();
      emit(U_CURC, v.r[1]);
      return v;
    }
    if (s == "phaseOneResult") {
      v.t = T_P1R;
      v.r[0] = R();
      emit(U_P1R, v.r[0]);
      const int z = ldi(0);
      v.nil = R();
      emit(U_EQ, v.nil, v.r[0], z);
      return v;
    }
    if (s == "compactorState") {
      v.t = T_MV;
      reg1(U_PHASE);
      return v;
    }
    if (s == "compactionHorizon") return reg1(U_HZ), v;
    if (s == "compactedTopicContext") return reg1(U_CTX), v;
    if (s == "crashTimes") return reg1(U_CRASH), v;
    if (s == "consumeTimes") {  // never assigned: the constant 0 of Init (model.h)
      v.r[0] = ldi(0);
      return v;
    }
    auto int_const = [&](long long x) {
      v.t = T_INT;
      v.r[0] = ldi(x);
      return v;
    };
    auto bool_const = [&](bool x) {
      v.t = T_BOOL;
      v.r[0] = ldi(x ? 1 : 0);
      return v;
    };
    if (s == "MessageSentLimit") return int_const(L_.N);
    if (s == "CompactionTimesLimit") return int_const(L_.C);
    if (s == "MaxCrashTimes") return int_const(L_.K);
    if (s == "ConsumeTimesLimit") return int_const(L_.ctl);
    if (s == "ModelConsumer") return bool_const(L_.consumer);
    if (s == "ModelProducer") return bool_const(L_.producer);
    if (s == "RetainNullKey") return bool_const(L_.retain);
    if (s == "Nil") {
      v.t = T_MV;
      v.r[0] = ldi(UV_NIL);
      v.nil_literal = true;
      return v;
    }
    static const char* kPhases[] = {"Compactor_In_PhaseOne", "Compactor_In_PhaseTwoWrite",
                                    "Compactor_In_PhaseTwoUpdateContext", "Compactor_In_PhaseTwoUpdateHorizon",
                                    "Compactor_In_PhaseTwoPersistCusror", "Compactor_In_PhaseTwoDeleteLedger"};
    for (int i = 0; i < 6; ++i)
      if (s == kPhases[i]) {
        v.t = T_MV;
        v.r[0] = ldi(UV_PHASE0 + i);
        return v;
      }
    if (s == "KeySpace" || s == "ValueSpace" || s == "Nat" || s == "Int" || s == "BOOLEAN") {
      v.t = T_SET;
      v.node = n;
      return v;
    }
    fail(n, "unknown identifier " + s);
  }

  // ---- lowering: every expression's value ends in the lowest free
  // registers (its temporaries are released), so a program needs about as
  // many registers as its expressions nest deep
  Val lower(const NodeP& n, const EnvP& env) {
    const int mark = nreg_;
    return compact(lower_(n, env), mark);
  }
  Val compact(Val v, int mark) {
    std::vector<int*> regs;
    for (int i = 0; i < 4; ++i)
      if (v.r[i] >= mark) regs.push_back(&v.r[i]);
    if (v.nil >= mark) regs.push_back(&v.nil);
    std::sort(regs.begin(), regs.end(), [](int* a, int* b) { return *a < *b; });
    int next = mark, last_src = -1;
    for (int* r : regs) {
      if (*r == last_src) {  // (a register shared by two fields)
        *r = next - 1;
        continue;
      }
      last_src = *r;
      if (*r != next) emit(U_MOV, next, *r);  // ascending: a target never clobbers a later source
      *r = next++;
    }
    nreg_ = next;
    return v;
  }
  Val lower_(const NodeP& n, const EnvP& env) {
    if (++depth_ > 200) fail(n, "definitions nest too deeply (recursive operators are not supported)");
    struct Guard { int& d; ~Guard() { --d; } } g{depth_};
    switch (n->k) {
      case Node::NUM: {
        if (n->v > 0x7fffffff) fail(n, "integer too large");
        Val v;
        v.r[0] = ldi(n->v);
        return v;
      }
      case Node::BOOL: {
        Val v;
        v.t = T_BOOL;
        v.r[0] = ldi(n->v);
        return v;
      }
      case Node::STR: fail(n, "strings are not values of this spec's numeric model");
      case Node::ID: return name(n, env, {});
      case Node::OPAPP: return opapp(n, env);
      case Node::UN: {
        if (n->s == "~") {
          const int a = boolean(n->c[0], env);
          Val v;
          v.t = T_BOOL;
          v.r[0] = R();
          emit(U_NOT, v.r[0], a);
          return v;
        }
        const int a = integer(n->c[0], env);
        Val v;
        v.r[0] = R();
        emit(U_NEG, v.r[0], a);
        return v;
      }
      case Node::BIN: return binary(n, env);
      case Node::JUNCT: return junction(n->s, n->c, env);
      case Node::IF: {
        const int c = boolean(n->c[0], env);
        const Val ta = probe(n->c[1], env), tb = probe(n->c[2], env);
        Val res = joined(n, ta, tb);
        const int j = emit(U_JZ, c);
        move_into(res, lower(n->c[1], env), n);
        const int k = emit(U_JMP);
        patch(j, pc());
        move_into(res, lower(n->c[2], env), n);
        patch(k, pc());
        return res;
      }
      case Node::CASE: {
        // arms tried in order (TLC takes the first true guard); none true: an error
        Val res;
        bool typed = false;
        for (size_t i = 0; i + 1 < n->c.size(); i += 2) {
          const Val t = probe(n->c[i + 1], env);
          res = typed ? joined(n, res, t) : alloc_like(t);
          typed = true;
        }
        std::vector<int> ends;
        bool other = false;
        for (size_t i = 0; i + 1 < n->c.size(); i += 2) {
          if (!n->c[i]) {
            move_into(res, lower(n->c[i + 1], env), n);
            other = true;
            break;
          }
          const int c = boolean(n->c[i], env);
          const int j = emit(U_JZ, c);
          move_into(res, lower(n->c[i + 1], env), n);
          ends.push_back(emit(U_JMP));
          patch(j, pc());
        }
        if (!other) emit(U_ERR);
        for (int e : ends) patch(e, pc());
        return res;
      }
      case Node::LET: {
        EnvP e = std::make_shared<Env>();
        e->up = env;
        for (size_t i = 0; i < n->names.size(); ++i) {
          Bind b;
          b.node = n->c[i];
          b.own_env = true;  // (LET definitions see each other, and themselves: recursion fails by depth)
          b.params = n->params[i];
          e->m[n->names[i]] = b;
        }
        return lower(n->c.back(), e);
      }
      case Node::QUANT: return quantifier(n, env, 0);
      case Node::CHOOSE: return choose(n, env);
      case Node::SETENUM:
      case Node::SETFILTER:
      case Node::SETMAP:
      case Node::RECSET: {
        Val v;
        v.t = T_SET;
        v.node = n;
        v.env = env;
        return v;
      }
      case Node::FCTOR: {
        Val v;
        v.t = T_FUNC;
        v.node = n;
        v.env = env;
        return v;
      }
      case Node::DOMAIN: {
        Val v;
        v.t = T_SET;
        v.node = n;
        v.env = env;
        return v;
      }
      case Node::APP: return apply(n, env);
      case Node::FIELD: return field(n, env);
      case Node::RECORD: return record(n, env);
      case Node::TUPLE: {
        if (!n->c.empty()) fail(n, "only the empty sequence << >> is supported as a tuple");
        Val v;
        v.t = T_SEQ;
        v.r[0] = ldi(0);
        return v;
      }
    }
    fail(n, "unsupported expression");
  }

  // an identifier (or operator application) in scope
  Val name(const NodeP& n, const EnvP& env, const std::vector<NodeP>& args) {
    const Env* owner = nullptr;
    if (const Bind* b = env->find(n->s, &owner)) {
      if (!b->by_name) {
        if (!args.empty()) fail(n, n->s + " takes no arguments");
        return b->v;
      }
      const EnvP benv = b->own_env ? std::const_pointer_cast<Env>(owner->shared_from_this()) : b->env;
      return substitute(n, b->node, benv, b->params, args, env);
    }
    auto it = defs.find(n->s);
    if (it != defs.end()) {
      NodeP body = body_of(it->second);
      return substitute(n, body, std::make_shared<Env>(), it->second.params, args, env);
    }
    if (!args.empty()) fail(n, "unknown operator " + n->s);
    return var_or_const(n);
  }

  Val substitute(const NodeP& at, const NodeP& body, const EnvP& benv, const std::vector<std::string>& params,
                 const std::vector<NodeP>& args, const EnvP& callenv) {
    if (params.size() != args.size())
      fail(at, at->s + " takes " + std::to_string(params.size()) + " argument(s), not " + std::to_string(args.size()));
    if (params.empty()) return lower(body, benv);
    EnvP e = std::make_shared<Env>();
    e->up = benv;
    for (size_t i = 0; i < params.size(); ++i) {
      Bind b;
      b.node = args[i];
      b.env = callenv;
      e->m[params[i]] = b;
    }
    return lower(body, e);
  }

  Val opapp(const NodeP& n, const EnvP& env) {
    const std::string& s = n->s;
    if (!env->find(s) && !defs.count(s)) {
      if (s == "Len") return length(n, env);
      if (s == "Cardinality") {
        Val v;
        v.r[0] = cardinality(n->c.at(0), env);
        return v;
      }
      if (s == "Head") {  // Head(s) = s[1]
        Node app = *n;
        auto one = std::make_shared<Node>();
        one->k = Node::NUM;
        one->v = 1;
        auto a = std::make_shared<Node>(app);
        a->k = Node::APP;
        a->c = {n->c.at(0), one};
        return apply(a, env);
      }
      fail(n, "operator " + s + " is not supported");
    }
    NodeP id = std::make_shared<Node>(*n);
    id->k = Node::ID;
    return name(id, env, n->c);
  }

  int boolean(const NodeP& n, const EnvP& env) {
    const Val v = lower(n, env);
    if (v.t != T_BOOL) fail(n, std::string("a boolean was expected, not a ") + tk_name(v.t));
    return v.r[0];
  }
  int integer(const NodeP& n, const EnvP& env) {
    const Val v = lower(n, env);
    if (v.t != T_INT) fail(n, std::string("an integer was expected, not a ") + tk_name(v.t));
    return v.r[0];
  }

  // registers for a value of v's type
  Val alloc_like(const Val& v) {
    Val r = v;
    for (int i = 0; i < 4; ++i)
      if (v.r[i] >= 0) r.r[i] = R();
    if (v.nil >= 0) r.nil = R();
    r.nil_literal = false;
    return r;
  }
  // the type of IF a THEN x ELSE y: equal types, or a composite and Nil
  Val joined(const NodeP& n, const Val& a, const Val& b) {
    auto composite = [](TK t) { return t == T_MSG || t == T_SEQ || t == T_CUR || t == T_P1R; };
    if (a.t == b.t && a.t != T_SET && a.t != T_FUNC && a.t != T_LEDGERS && a.t != T_LFK) {
      Val r = alloc_like(a);
      if (r.nil < 0 && b.nil >= 0) r.nil = R();
      return r;
    }
    if (a.t == T_MV && a.nil_literal && composite(b.t)) {
      Val r = alloc_like(b);
      if (r.nil < 0) r.nil = R();
      return r;
    }
    if (b.t == T_MV && b.nil_literal && composite(a.t)) {
      Val r = alloc_like(a);
      if (r.nil < 0) r.nil = R();
      return r;
    }
    fail(n, std::string("branches of different types: ") + tk_name(a.t) + " and " + tk_name(b.t));
  }
  void move_into(const Val& dst, const Val& src, const NodeP& n) {
    if (src.t == T_MV && src.nil_literal && dst.t != T_MV) {  // Nil into a composite
      emit(U_LDI, dst.nil, 0, 0, 1);
      return;
    }
    if (src.t != dst.t) fail(n, "branches of different types");
    for (int i = 0; i < 4; ++i)
      if (dst.r[i] >= 0) emit(U_MOV, dst.r[i], src.r[i]);
    if (dst.nil >= 0) {
      if (src.nil >= 0) emit(U_MOV, dst.nil, src.nil);
      else emit(U_LDI, dst.nil, 0, 0, 0);
    }
  }

  Val junction(const std::string& op, const std::vector<NodeP>& items, const EnvP& env) {
    // /\: FALSE at the first false item; \/: TRUE at the first true one (left to right, as TLC)
    Val v;
    v.t = T_BOOL;
    v.r[0] = R();
    const bool conj = op == "/\\";
    std::vector<int> exits;
    for (const NodeP& it : items) {
      const int mark = nreg_;
      const int b = boolean(it, env);
      emit(U_MOV, v.r[0], b);
      exits.push_back(emit(conj ? U_JZ : U_JNZ, v.r[0]));
      nreg_ = mark;
    }
    for (int e : exits) patch(e, pc());
    return v;
  }

  Val binary(const NodeP& n, const EnvP& env) {
    const std::string& op = n->s;
    if (op == "/\\" || op == "\\/") return junction(op, {n->c[0], n->c[1]}, env);
    if (op == "=>") {
      Val v;
      v.t = T_BOOL;
      v.r[0] = R();
      const int a = boolean(n->c[0], env);
      emit(U_NOT, v.r[0], a);
      const int j = emit(U_JNZ, v.r[0]);
      const int b = boolean(n->c[1], env);
      emit(U_MOV, v.r[0], b);
      patch(j, pc());
      return v;
    }
    if (op == "<=>") {
      const int a = boolean(n->c[0], env), b = boolean(n->c[1], env);
      Val v;
      v.t = T_BOOL;
      v.r[0] = R();
      emit(U_EQ, v.r[0], a, b);
      return v;
    }
    if (op == "=" || op == "#") {
      const Val a = lower(n->c[0], env), b = lower(n->c[1], env);
      Val v;
      v.t = T_BOOL;
      v.r[0] = equal(n, a, b);
      if (op == "#") emit(U_NOT, v.r[0], v.r[0]);
      return v;
    }
    if (op == "\\in" || op == "\\notin") {
      const Val x = lower(n->c[0], env);
      const Val s = lower(n->c[1], env);
      if (s.t != T_SET && s.t != T_SEQ) fail(n, std::string("\\in needs a set, not a ") + tk_name(s.t));
      if (s.t != T_SET) fail(n, "\\in a sequence is not set membership");
      Val v;
      v.t = T_BOOL;
      v.r[0] = member(n, x, s);
      if (op == "\\notin") emit(U_NOT, v.r[0], v.r[0]);
      return v;
    }
    if (op == "\\subseteq") {  // \A x \in A : x \in B
      const Val a = lower(n->c[0], env), b = lower(n->c[1], env);
      if (a.t != T_SET || b.t != T_SET) fail(n, "\\subseteq needs sets");
      Val v;
      v.t = T_BOOL;
      v.r[0] = R();
      emit(U_LDI, v.r[0], 0, 0, 1);
      std::vector<int> exits;
      iterate(n, a, [&](const Val& x) {
        const int m = member(n, x, b);
        emit(U_MOV, v.r[0], m);
        exits.push_back(emit(U_JZ, v.r[0]));
      });
      for (int e : exits) patch(e, pc());
      return v;
    }
    if (op == "\\cup" || op == "\\cap" || op == "\\" || op == "..") {
      Val v;
      v.t = T_SET;
      v.node = n;
      v.env = env;
      return v;
    }
    // arithmetic and order on integers
    const int a = integer(n->c[0], env), b = integer(n->c[1], env);
    Val v;
    v.r[0] = R();
    if (op == "+") emit(U_ADD, v.r[0], a, b);
    else if (op == "-") emit(U_SUB, v.r[0], a, b);
    else if (op == "*") emit(U_MUL, v.r[0], a, b);
    else if (op == "\\div" || op == "%") {
      const int z = ldi(0), c = R();
      emit(op == "%" ? U_LT : U_EQ, c, op == "%" ? z : b, op == "%" ? b : z);  // %: 0 < b; \div: b = 0
      const int j = emit(op == "%" ? U_JNZ : U_JZ, c);
      emit(U_ERR);
      patch(j, pc());
      emit(op == "%" ? U_MOD : U_DIV, v.r[0], a, b);
    } else {
      v.t = T_BOOL;
      if (op == "<") emit(U_LT, v.r[0], a, b);
      else if (op == "<=") emit(U_LE, v.r[0], a, b);
      else if (op == ">") emit(U_LT, v.r[0], b, a);
      else if (op == ">=") emit(U_LE, v.r[0], b, a);
      else fail(n, "unsupported operator " + op);
    }
    return v;
  }

  // x = y by type (TLC: an untyped model value equals only itself, and differs from every other value)
  int equal(const NodeP& n, const Val& a, const Val& b) {
    const int r = R();
    auto fields_equal = [&](int k) {
      emit(U_LDI, r, 0, 0, 1);
      for (int i = 0; i < k; ++i) {
        const int e = R();
        emit(U_EQ, e, a.r[i], b.r[i]);
        emit(U_AND, r, r, e);
      }
    };
    if (a.t == b.t && (a.t == T_INT || a.t == T_BOOL || a.t == T_MV)) {
      emit(U_EQ, r, a.r[0], b.r[0]);
      return r;
    }
    if (a.t == T_SET && b.t == T_SET) {  // A \subseteq B /\ B \subseteq A
      emit(U_LDI, r, 0, 0, 1);
      std::vector<int> exits;
      for (int dir = 0; dir < 2; ++dir) {
        const Val& x = dir ? b : a;
        const Val& y = dir ? a : b;
        iterate(n, x, [&](const Val& e) {
          const int m = member(n, e, y);
          emit(U_MOV, r, m);
          exits.push_back(emit(U_JZ, r));
        });
      }
      for (int e : exits) patch(e, pc());
      return r;
    }
    const bool ca = a.t == T_MSG || a.t == T_SEQ || a.t == T_CUR || a.t == T_P1R;
    const bool cb = b.t == T_MSG || b.t == T_SEQ || b.t == T_CUR || b.t == T_P1R;
    if (ca && b.t == T_MV) return nil_equal(a, b, r);
    if (cb && a.t == T_MV) return nil_equal(b, a, r);
    if ((a.t == T_MV && (b.t == T_INT || b.t == T_BOOL)) || (b.t == T_MV && (a.t == T_INT || a.t == T_BOOL))) {
      emit(U_LDI, r, 0, 0, 0);  // a model value differs from every integer and boolean
      return r;
    }
    if (a.t != b.t || !ca) fail(n, std::string("cannot compare a ") + tk_name(a.t) + " with a " + tk_name(b.t));
    const int k = a.t == T_MSG ? 3 : a.t == T_CUR ? 2 : 1;
    fields_equal(k);
    if (a.nil >= 0 || b.nil >= 0) {  // equal iff both Nil, or neither and the fields agree
      const int na = a.nil >= 0 ? a.nil : ldi(0), nb = b.nil >= 0 ? b.nil : ldi(0);
      const int both = R(), same = R(), none = R();
      emit(U_AND, both, na, nb);
      emit(U_EQ, same, na, nb);
      emit(U_OR, none, na, nb);
      emit(U_NOT, none, none);
      emit(U_AND, r, r, none);
      emit(U_OR, r, r, both);
      (void)same;
    }
    return r;
  }
  int nil_equal(const Val& comp, const Val& mv, int r) {
    // a composite equals a model value only if it is Nil and the model value is Nil
    if (comp.nil < 0) {
      emit(U_LDI, r, 0, 0, 0);
      return r;
    }
    const int isnil = R();
    const int k = ldi(UV_NIL);
    emit(U_EQ, isnil, mv.r[0], k);
    emit(U_AND, r, isnil, comp.nil);
    return r;
  }

  // e.f
  Val field(const NodeP& n, const EnvP& env) {
    const Val r = lower(n->c[0], env);
    const std::string& f = n->s;
    auto guard_nil = [&](const Val& v) {
      if (v.nil < 0) return;
      const int j = emit(U_JZ, v.nil);
      emit(U_ERR);  // a field of Nil
      patch(j, pc());
    };
    Val v;
    if (r.t == T_MSG && (f == "id" || f == "key" || f == "value")) {
      guard_nil(r);
      v.r[0] = r.r[f == "id" ? 0 : f == "key" ? 1 : 2];
      return v;
    }
    if (r.t == T_CUR && (f == "compactionHorizon" || f == "compactedTopicContext")) {
      guard_nil(r);
      v.r[0] = r.r[f == "compactionHorizon" ? 0 : 1];
      return v;
    }
    if (r.t == T_P1R && (f == "readPosition" || f == "latestForKey")) {
      guard_nil(r);
      if (f == "readPosition") {
        v.r[0] = r.r[0];
        return v;
      }
      v.t = T_LFK;
      v.r[0] = r.r[0];
      return v;
    }
    if (r.t == T_MV) {  // e.g. Nil.f: always an evaluation error when reached
      emit(U_ERR);
      fail(n, "field " + f + " of a model value");
    }
    fail(n, "no field " + f + " in a " + tk_name(r.t));
  }

  Val record(const NodeP& n, const EnvP& env) {
    std::map<std::string, NodeP> f;
    for (size_t i = 0; i < n->names.size(); ++i) f[n->names[i]] = n->c[i];
    Val v;
    if (f.size() == 3 && f.count("id") && f.count("key") && f.count("value")) {
      v.t = T_MSG;
      // TLC evaluates a record's fields in the order written
      std::map<std::string, int> reg;
      for (size_t i = 0; i < n->names.size(); ++i) reg[n->names[i]] = integer(n->c[i], env);
      v.r[0] = reg["id"];
      v.r[1] = reg["key"];
      v.r[2] = reg["value"];
      return v;
    }
    if (f.size() == 2 && f.count("compactionHorizon") && f.count("compactedTopicContext")) {
      v.t = T_CUR;
      std::map<std::string, int> reg;
      for (size_t i = 0; i < n->names.size(); ++i) reg[n->names[i]] = integer(n->c[i], env);
      v.r[0] = reg["compactionHorizon"];
      v.r[1] = reg["compactedTopicContext"];
      return v;
    }
    fail(n, "records other than [id, key, value] messages and the cursor are not supported");
  }

  // element j of a sequence value (mask of message positions): the message at the j-th set bit
  Val seq_elem(const Val& s, int j) {
    if (s.nil >= 0) {  // Nil[j]
      const int k = emit(U_JZ, s.nil);
      emit(U_ERR);
      patch(k, pc());
    }
    const int len = R(), ok = R(), one = ldi(1), c = R();
    emit(U_POPC, len, s.r[0]);
    emit(U_LE, ok, one, j);
    emit(U_LE, c, j, len);
    emit(U_AND, ok, ok, c);
    const int k = emit(U_JNZ, ok);
    emit(U_ERR);  // out of the sequence's domain
    patch(k, pc());
    Val m;
    m.t = T_MSG;
    m.r[0] = R();
    emit(U_NTH, m.r[0], s.r[0], j);  // the id is the message's position
    m.r[1] = R();
    emit(U_MKEY, m.r[1], m.r[0]);
    m.r[2] = R();
    emit(U_MVAL, m.r[2], m.r[0]);
    return m;
  }

  // f[x]
  Val apply(const NodeP& n, const EnvP& env) {
    const Val f = lower(n->c[0], env);
    if (f.t == T_SEQ) {
      const int j = integer(n->c[1], env);
      return seq_elem(f, j);
    }
    if (f.t == T_LEDGERS) {  // compactedLedgers[i]: 1..CompactionTimesLimit
      const int i = integer(n->c[1], env);
      in_range_or_error(i, 1, L_.C);
      Val s;
      s.t = T_SEQ;
      const int p = R();
      emit(U_LEDP, p, i);
      s.nil = R();
      emit(U_NOT, s.nil, p);
      s.r[0] = R();
      emit(U_LEDM, s.r[0], i);
      return s;
    }
    if (f.t == T_LFK) {  // latestForKey[k]: k in GetKeys(messages[1..readPosition]) \ {NullKey}
      const int k = integer(n->c[1], env);
      Val v;
      v.r[0] = R();
      emit(U_LFK, v.r[0], k, f.r[0]);
      const int z = ldi(0), ok = R(), nz = R();
      emit(U_NE, ok, v.r[0], z);
      emit(U_NE, nz, k, z);
      emit(U_AND, ok, ok, nz);
      const int j = emit(U_JNZ, ok);
      emit(U_ERR);
      patch(j, pc());
      return v;
    }
    if (f.t == T_FUNC) {  // [y \in S |-> e][x]: x must be in S
      const Val x = lower(n->c[1], env);
      const Val dom = lower(f.node->c[0], f.env);
      if (dom.t != T_SET) fail(n, "a function's domain must be a set");
      const int m = member(n, x, dom);
      const int j = emit(U_JNZ, m);
      emit(U_ERR);
      patch(j, pc());
      EnvP e = std::make_shared<Env>();
      e->up = f.env;
      Bind b;
      b.by_name = false;
      b.v = x;
      e->m[f.node->names[0]] = b;
      return lower(f.node->c[1], e);
    }
    fail(n, std::string("cannot apply a ") + tk_name(f.t));
  }

  void in_range_or_error(int x, int lo, int hi) {
    const int a = ldi(lo), b = ldi(hi), ok = R(), c = R();
    emit(U_LE, ok, a, x);
    emit(U_LE, c, x, b);
    emit(U_AND, ok, ok, c);
    const int j = emit(U_JNZ, ok);
    emit(U_ERR);
    patch(j, pc());
  }

  Val length(const NodeP& n, const EnvP& env) {
    const Val s = lower(n->c.at(0), env);
    Val v;
    if (s.t == T_SEQ) {
      if (s.nil >= 0) {  // Len(Nil)
        const int k = emit(U_JZ, s.nil);
        emit(U_ERR);
        patch(k, pc());
      }
      v.r[0] = R();
      emit(U_POPC, v.r[0], s.r[0]);
      return v;
    }
    if (s.t == T_LEDGERS) {
      v.r[0] = ldi(L_.C);
      return v;
    }
    if (s.t == T_FUNC) {
      // Len of [i \in 1..n |-> e]: TLC enumerates the function (every e is evaluated), then n
      const NodeP dom = s.node->c[0];
      const Val d = lower(dom, s.env);
      if (d.t != T_SET || !(d.node->k == Node::BIN && d.node->s == "..")) fail(n, "Len of a function needs domain 1..n");
      const int lo = integer(d.node->c[0], d.env), hi = integer(d.node->c[1], d.env);
      const int one = ldi(1), ok = R(), e = R();
      emit(U_EQ, ok, lo, one);
      const int le = R();
      emit(U_LT, le, hi, lo);  // an empty domain is 1..0 too
      emit(U_OR, ok, ok, le);
      const int j = emit(U_JNZ, ok);
      emit(U_ERR);  // not a sequence
      patch(j, pc());
      iterate(n, d, [&](const Val& x) {
        EnvP en = std::make_shared<Env>();
        en->up = s.env;
        Bind b;
        b.by_name = false;
        b.v = x;
        en->m[s.node->names[0]] = b;
        const int mark = nreg_;
        lower(s.node->c[1], en);
        nreg_ = mark;
      });
      v.r[0] = R();
      emit(U_SUB, e, hi, lo);
      emit(U_ADDI, v.r[0], e, 0, 1);
      const int z = ldi(0), neg = R();
      emit(U_LT, neg, v.r[0], z);
      const int k = emit(U_JZ, neg);
      emit(U_LDI, v.r[0], 0, 0, 0);
      patch(k, pc());
      return v;
    }
    fail(n, std::string("Len of a ") + tk_name(s.t));
  }

  // ---- sets: never built; consumers iterate them or test membership
  // iterate: emits a loop over the set's elements (TLC's order for integer
  // sets: ascending), calling body with each element in registers
  void iterate(const NodeP& at, const Val& s, const std::function<void(const Val&)>& body) {
    const NodeP n = s.node;
    const EnvP env = s.env;
    if (n->k == Node::ID || n->k == Node::OPAPP) {  // KeySpace / ValueSpace (KeySet, ... resolve through their defs)
      const std::string& nm = n->s;
      if (nm == "KeySpace" || nm == "ValueSpace") {
        const bool keys = nm == "KeySpace";
        const int cnt = keys ? P_->nk : P_->nv;
        const int i = R(), lim = ldi(cnt), c = R(), z = ldi(0);
        emit(U_LDI, i, 0, 0, 0);
        const int top = pc();
        emit(U_LT, c, i, lim);
        const int j = emit(U_JZ, c);
        Val x;
        x.r[0] = R();
        emit(U_KAT, x.r[0], i, 0, keys ? 0 : 1);
        const int isz = R();
        emit(U_EQ, isz, x.r[0], z);  // NullKey / NullValue belong to KeySet, not KeySpace
        const int skip = emit(U_JNZ, isz);
        const int mark = nreg_;
        body(x);
        nreg_ = mark;
        patch(skip, pc());
        emit(U_ADDI, i, i, 0, 1);
        emit(U_JMP, 0, 0, 0, top);
        patch(j, pc());
        return;
      }
      if (nm == "BOOLEAN") {
        for (int b = 0; b < 2; ++b) {
          Val x;
          x.t = T_BOOL;
          x.r[0] = ldi(b);
          const int mark = nreg_;
          body(x);
          nreg_ = mark;
        }
        return;
      }
      fail(at, nm + " is not enumerable");
    }
    if (n->k == Node::BIN && n->s == "..") {
      const int lo = integer(n->c[0], env), hi = integer(n->c[1], env);
      const int i = R(), c = R();
      emit(U_MOV, i, lo);
      const int top = pc();
      emit(U_LE, c, i, hi);
      const int j = emit(U_JZ, c);
      Val x;
      x.r[0] = i;
      const int mark = nreg_;
      body(x);
      nreg_ = mark;
      emit(U_ADDI, i, i, 0, 1);
      emit(U_JMP, 0, 0, 0, top);
      patch(j, pc());
      return;
    }
    if (n->k == Node::SETENUM) {
      // TLC normalizes an enumerated set: sorted, duplicates removed.  Elements
      // are visited as written; each is skipped if an earlier one equals it,
      // which is order-insensitive for \A, \E, membership and counting;
      // CHOOSE takes the least element itself (choose()).
      std::vector<Val> els;
      for (const NodeP& e : n->c) els.push_back(lower(e, env));
      for (size_t i = 0; i < els.size(); ++i) {
        std::vector<int> skips;
        for (size_t k = 0; k < i; ++k) skips.push_back(emit(U_JNZ, equal(at, els[k], els[i])));
        const int mark = nreg_;
        body(els[i]);
        nreg_ = mark;
        for (int sk : skips) patch(sk, pc());
      }
      return;
    }
    if (n->k == Node::SETFILTER) {  // {y \in S : P}
      const Val base = lower(n->c[0], env);
      if (base.t != T_SET) fail(at, "a filter needs a set");
      iterate(at, base, [&](const Val& y) {
        EnvP e = bind1(env, n->names[0], y);
        const int p = boolean(n->c[1], e);
        const int j = emit(U_JZ, p);
        body(y);
        patch(j, pc());
      });
      return;
    }
    if (n->k == Node::SETMAP) {  // {e : y \in S}: duplicates visited once (as TLC's normalized set)
      map_iterate(at, n, env, 0, env, body);
      return;
    }
    if (n->k == Node::BIN && (n->s == "\\cup" || n->s == "\\cap" || n->s == "\\")) {
      const Val a = lower(n->c[0], env), b = lower(n->c[1], env);
      if (a.t != T_SET || b.t != T_SET) fail(at, "set operators need sets");
      if (n->s == "\\cup") {
        iterate(at, a, body);
        iterate(at, b, [&](const Val& x) {  // the elements of B not in A
          const int m = member(at, x, a);
          const int j = emit(U_JNZ, m);
          body(x);
          patch(j, pc());
        });
      } else {
        const bool inter = n->s == "\\cap";
        iterate(at, a, [&](const Val& x) {
          const int m = member(at, x, b);
          const int j = emit(inter ? U_JZ : U_JNZ, m);
          body(x);
          patch(j, pc());
        });
      }
      return;
    }
    if (n->k == Node::DOMAIN) {
      const Val f = lower(n->c[0], env);
      if (f.t == T_SEQ) {
        if (f.nil >= 0) {
          const int k = emit(U_JZ, f.nil);
          emit(U_ERR);  // DOMAIN Nil
          patch(k, pc());
        }
        const int len = R();
        emit(U_POPC, len, f.r[0]);
        range_loop(ldi(1), len, body);
        return;
      }
      if (f.t == T_LEDGERS) {
        range_loop(ldi(1), ldi(L_.C), body);
        return;
      }
      if (f.t == T_FUNC) {
        const Val d = lower(f.node->c[0], f.env);
        iterate(at, d, body);
        return;
      }
      if (f.t == T_LFK) {  // GetKeys(messages[1..r]) \ {NullKey}: first occurrences of non-null keys
        const int p = R(), c = R(), z = ldi(0);
        emit(U_LDI, p, 0, 0, 1);
        const int top = pc();
        emit(U_LE, c, p, f.r[0]);
        const int j = emit(U_JZ, c);
        Val x;
        x.r[0] = R();
        emit(U_MKEY, x.r[0], p);
        const int isz = R();
        emit(U_EQ, isz, x.r[0], z);
        const int skip0 = emit(U_JNZ, isz);
        const int last = R();  // latest position of this key up to r: the key is first seen at p iff ...
        emit(U_LFK, last, x.r[0], p);  // ... the latest position within 1..p is p and none before
        const int q = R(), prev = R();
        emit(U_ADDI, q, p, 0, -1);
        emit(U_LFK, prev, x.r[0], q);
        const int seen = R();
        emit(U_NE, seen, prev, z);
        const int skip1 = emit(U_JNZ, seen);
        const int mark = nreg_;
        body(x);
        nreg_ = mark;
        patch(skip0, pc());
        patch(skip1, pc());
        emit(U_ADDI, p, p, 0, 1);
        emit(U_JMP, 0, 0, 0, top);
        patch(j, pc());
        return;
      }
      fail(at, std::string("DOMAIN of a ") + tk_name(f.t));
    }
    if (n->k == Node::RECSET) fail(at, "a record set is only supported on the right of \\in");
    fail(at, "this set cannot be enumerated");
  }

  void range_loop(int lo, int hi, const std::function<void(const Val&)>& body) {
    const int i = R(), c = R();
    emit(U_MOV, i, lo);
    const int top = pc();
    emit(U_LE, c, i, hi);
    const int j = emit(U_JZ, c);
    Val x;
    x.r[0] = i;
    const int mark = nreg_;
    body(x);
    nreg_ = mark;
    emit(U_ADDI, i, i, 0, 1);
    emit(U_JMP, 0, 0, 0, top);
    patch(j, pc());
  }

  // {e : y1 \in S1, y2 \in S2, ..}: bound variables k.. nest; each image is
  // visited once: skipped when an earlier binding gave an equal image
  void map_iterate(const NodeP& at, const NodeP& n, const EnvP& env, size_t k, const EnvP& bound,
                   const std::function<void(const Val&)>& body) {
    if (k < n->names.size()) {
      const Val s = lower(n->c[1 + k], env);
      if (s.t != T_SET) fail(at, "a set map ranges over sets");
      // a counter of the bindings visited so far orders them for the duplicate test
      iterate(at, s, [&](const Val& y) { map_iterate(at, n, env, k + 1, bind1(bound, n->names[k], y), body); });
      return;
    }
    const Val img = lower(n->c[0], bound);
    // earlier bindings: re-enumerate and stop at the current one (by image equality of all earlier ones)
    const int dup = R();
    emit(U_LDI, dup, 0, 0, 0);
    std::vector<int> done;
    earlier_images(at, n, env, 0, env, bound, img, dup, &done);
    for (int d : done) patch(d, pc());
    const int j = emit(U_JNZ, dup);
    const int mark = nreg_;
    body(img);
    nreg_ = mark;
    patch(j, pc());
  }
  // sets dup = 1 if a binding before the current one (lexicographic over the
  // bound variables' enumeration) has an image equal to img
  void earlier_images(const NodeP& at, const NodeP& n, const EnvP& env, size_t k, const EnvP& bound,
                      const EnvP& current, const Val& img, int dup, std::vector<int>* done) {
    if (k < n->names.size()) {
      const Val s = lower(n->c[1 + k], env);
      iterate(at, s, [&](const Val& y) {
        EnvP b = bind1(bound, n->names[k], y);
        // reaching the current binding: nothing before it remains
        const Bind* cur = current->find(n->names[k]);
        const int same = equal(at, y, cur->v);
        if (k + 1 == n->names.size()) {
          done->push_back(emit(U_JNZ, same));
          const Val other = lower(n->c[0], b);
          const int e = equal(at, other, img);
          emit(U_OR, dup, dup, e);
        } else {
          // a prefix equal to the current one: recurse; a smaller one: every completion is earlier
          earlier_images(at, n, env, k + 1, b, current, img, dup, done);
        }
      });
      return;
    }
  }

  EnvP bind1(const EnvP& env, const std::string& name, const Val& v) {
    EnvP e = std::make_shared<Env>();
    e->up = env;
    Bind b;
    b.by_name = false;
    b.v = v;
    e->m[name] = b;
    return e;
  }

  // x \in S (TLC: without enumerating S where it can)
  int member(const NodeP& at, const Val& x, const Val& s) {
    const NodeP n = s.node;
    const EnvP env = s.env;
    const int r = R();
    if (n->k == Node::ID) {
      const std::string& nm = n->s;
      if (nm == "Nat" || nm == "Int") {
        if (x.t != T_INT) {
          emit(U_LDI, r, 0, 0, 0);
          return r;
        }
        if (nm == "Int") {
          emit(U_LDI, r, 0, 0, 1);
        } else {
          const int z = ldi(0);
          emit(U_LE, r, z, x.r[0]);
        }
        return r;
      }
      if (nm == "BOOLEAN") {
        emit(U_LDI, r, 0, 0, x.t == T_BOOL ? 1 : 0);
        return r;
      }
    }
    if (n->k == Node::BIN && n->s == "..") {
      const int lo = integer(n->c[0], env), hi = integer(n->c[1], env);
      if (x.t != T_INT) fail(at, std::string("is a ") + tk_name(x.t) + " in an integer interval?");
      const int c = R();
      emit(U_LE, r, lo, x.r[0]);
      emit(U_LE, c, x.r[0], hi);
      emit(U_AND, r, r, c);
      return r;
    }
    if (n->k == Node::SETFILTER) {  // x \in S /\ P(x)
      const Val base = lower(n->c[0], env);
      const int m = member(at, x, base);
      emit(U_MOV, r, m);
      const int j = emit(U_JZ, r);
      EnvP e = bind1(env, n->names[0], x);
      const int p = boolean(n->c[1], e);
      emit(U_MOV, r, p);
      patch(j, pc());
      return r;
    }
    if (n->k == Node::BIN && (n->s == "\\cup" || n->s == "\\cap" || n->s == "\\")) {
      const Val a = lower(n->c[0], env), b = lower(n->c[1], env);
      const int ma = member(at, x, a);
      emit(U_MOV, r, ma);
      // \cup: A or B; \cap: A and B; \: A and not B (left to right)
      const int j = emit(n->s == "\\cup" ? U_JNZ : U_JZ, r);
      const int mb = member(at, x, b);
      if (n->s == "\\") emit(U_NOT, r, mb);
      else emit(U_MOV, r, mb);
      patch(j, pc());
      return r;
    }
    if (n->k == Node::RECSET) {  // [f1 : S1, ..]: a record with exactly these fields, each in its set
      std::map<std::string, NodeP> f;
      for (size_t i = 0; i < n->names.size(); ++i) f[n->names[i]] = n->c[i];
      std::vector<std::pair<std::string, int>> regs;
      if (x.t == T_MSG && f.size() == 3 && f.count("id") && f.count("key") && f.count("value")) {
        regs = {{"id", x.r[0]}, {"key", x.r[1]}, {"value", x.r[2]}};
      } else if (x.t == T_CUR && f.size() == 2 && f.count("compactionHorizon") && f.count("compactedTopicContext")) {
        regs = {{"compactionHorizon", x.r[0]}, {"compactedTopicContext", x.r[1]}};
      } else if (x.t == T_MV || x.t == T_MSG || x.t == T_CUR || x.t == T_INT || x.t == T_SEQ || x.t == T_P1R) {
        emit(U_LDI, r, 0, 0, 0);  // not a record of these fields
        return r;
      } else {
        fail(at, "unsupported record-set membership");
      }
      if (x.nil >= 0) emit(U_NOT, r, x.nil);
      else emit(U_LDI, r, 0, 0, 1);
      std::vector<int> exits;
      exits.push_back(emit(U_JZ, r));
      for (auto& fr : regs) {
        Val fv;
        fv.r[0] = fr.second;
        const Val s2 = lower(f[fr.first], env);
        if (s2.t != T_SET) fail(at, "a record set's fields range over sets");
        const int m = member(at, fv, s2);
        emit(U_MOV, r, m);
        exits.push_back(emit(U_JZ, r));
      }
      for (int e : exits) patch(e, pc());
      return r;
    }
    if (n->k == Node::ID && (n->s == "KeySpace" || n->s == "ValueSpace") && x.t == T_INT) {
      // KeySet / ValueSet without NullKey / NullValue (0)
      const int z = ldi(0), nz = R();
      emit(U_KIN, r, x.r[0], 0, n->s == "KeySpace" ? 0 : 1);
      emit(U_NE, nz, x.r[0], z);
      emit(U_AND, r, r, nz);
      return r;
    }
    // general: \E y \in S : y = x
    emit(U_LDI, r, 0, 0, 0);
    std::vector<int> exits;
    iterate(at, s, [&](const Val& y) {
      const int e = equal(at, y, x);
      emit(U_MOV, r, e);
      exits.push_back(emit(U_JNZ, r));
    });
    for (int e : exits) patch(e, pc());
    return r;
  }

  int cardinality(const NodeP& sn, const EnvP& env) {
    const Val s = lower(sn, env);
    if (s.t != T_SET) fail(sn, "Cardinality of a non-set");
    const int cnt = R();
    emit(U_LDI, cnt, 0, 0, 0);
    iterate(sn, s, [&](const Val&) { emit(U_ADDI, cnt, cnt, 0, 1); });
    return cnt;
  }

  // \A / \E x \in S, ... : P -- TLC enumerates S (evaluating every element) before testing P
  Val quantifier(const NodeP& n, const EnvP& env, size_t k) {
    const bool all = n->s == "A";
    Val v;
    v.t = T_BOOL;
    v.r[0] = R();
    emit(U_LDI, v.r[0], 0, 0, all ? 1 : 0);
    std::vector<int> exits;
    std::function<void(size_t, const EnvP&)> nest = [&](size_t i, const EnvP& e) {
      if (i == n->names.size()) {
        const int p = boolean(n->c.back(), e);
        emit(U_MOV, v.r[0], p);
        exits.push_back(emit(all ? U_JZ : U_JNZ, v.r[0]));
        return;
      }
      const Val s = lower(n->c[i], e);
      if (s.t != T_SET) fail(n, "a quantifier ranges over a set");
      force(n, s);
      iterate(n, s, [&](const Val& x) { nest(i + 1, bind1(e, n->names[i], x)); });
    };
    (void)k;
    nest(0, env);
    for (int e : exits) patch(e, pc());
    return v;
  }

  // evaluates every element of a set whose elements can fail (TLC builds the set first)
  void force(const NodeP& at, const Val& s) {
    if (!can_fail(s.node)) return;
    if (s.node->k == Node::BIN && s.node->s == "..") {  // a range's elements cannot fail once its bounds are known
      integer(s.node->c[0], s.env);
      integer(s.node->c[1], s.env);
      return;
    }
    const int n0 = P_->n_ins, nr = nreg_;
    iterate(at, s, [&](const Val&) {});
    // a loop none of whose elements can fail is dropped: the set's own
    // evaluation (its failures included) is repeated by the iteration that
    // follows, and an empty loop only costs the check its time
    if (!loop_can_fail(n0, P_->n_ins)) {
      P_->n_ins = n0;
      nreg_ = nr;
    }
  }
  // whether the code [n0, n) holds a loop (a backward jump and its target)
  // that can fail: an error-raising instruction inside it, or a jump from
  // inside it to somewhere other than the loop or its exit
  bool loop_can_fail(int n0, int n) const {
    auto jump = [](uint8_t op) { return op == U_JMP || op == U_JZ || op == U_JNZ; };
    auto raises = [](uint8_t op) {
      return op == U_ERR || op == U_ADD || op == U_SUB || op == U_MUL || op == U_NEG || op == U_DIV ||
             op == U_MOD || op == U_RET;
    };
    for (int j = n0; j < n; ++j) {
      const UInsn& b = P_->ins[j];
      if (!jump(b.op) || b.imm > j) continue;
      if (b.imm < n0) return true;
      for (int k = b.imm; k <= j; ++k) {
        const UInsn& in = P_->ins[k];
        if (raises(in.op)) return true;
        if (jump(in.op) && (in.imm < b.imm || in.imm > j + 1)) return true;
      }
    }
    return false;
  }
  static bool can_fail(const NodeP& n) {
    if (!n) return false;
    if (n->k == Node::ID || n->k == Node::NUM || n->k == Node::BOOL) return false;
    if (n->k == Node::BIN && n->s == "..") return can_fail(n->c[0]) || can_fail(n->c[1]);
    return true;
  }

  // CHOOSE x \in S : P -- TLC takes the first element of the normalized (sorted) set: the least integer
  Val choose(const NodeP& n, const EnvP& env) {
    const Val s = lower(n->c[0], env);
    if (s.t != T_SET) fail(n, "CHOOSE ranges over a set");
    const Val t = probe_elem(n, s);
    if (t.t != T_INT) fail(n, "CHOOSE is supported over sets of integers");
    force(n, s);
    Val v;
    v.r[0] = R();
    const int found = R();
    emit(U_LDI, found, 0, 0, 0);
    iterate(n, s, [&](const Val& x) {
      EnvP e = bind1(env, n->names[0], x);
      const int p = boolean(n->c[1], e);
      const int j = emit(U_JZ, p);
      // keep the least
      const int better = R();
      emit(U_LT, better, x.r[0], v.r[0]);
      const int nf = R();
      emit(U_NOT, nf, found);
      emit(U_OR, better, better, nf);
      const int k = emit(U_JZ, better);
      emit(U_MOV, v.r[0], x.r[0]);
      emit(U_LDI, found, 0, 0, 1);
      patch(k, pc());
      patch(j, pc());
    });
    const int j = emit(U_JNZ, found);
    emit(U_ERR);  // no element satisfies P
    patch(j, pc());
    return v;
  }

  Val probe_elem(const NodeP& at, const Val& s) {
    const int n_ins = P_->n_ins, nr = nreg_;
    Val t;
    bool got = false;
    ++dry_;
    try {
      iterate(at, s, [&](const Val& x) {
        if (!got) t = x;
        got = true;
      });
    } catch (...) {
      --dry_;
      P_->n_ins = n_ins;
      nreg_ = nr;
      throw;
    }
    --dry_;
    P_->n_ins = n_ins;
    nreg_ = nr;
    if (!got) t.t = T_INT;
    return t;
  }
};

std::vector<Def> split_defs(const std::string& text) {
  std::vector<Def> out;
  std::istringstream in(text);
  std::string line;
  int ln = 0;
  Def* cur = nullptr;
  while (std::getline(in, line)) {
    ++ln;
    if (line.compare(0, 6, "@@DEF ") == 0) {
      std::istringstream h(line.substr(6));
      Def d;
      h >> d.name;
      for (std::string p; h >> p;) {
        if (p.compare(0, 1, "@") == 0) {
          d.line0 = std::atoi(p.c_str() + 1);
          continue;
        }
        d.params.push_back(p);
      }
      if (!d.line0) d.line0 = ln + 1;
      out.push_back(d);
      cur = &out.back();
      continue;
    }
    if (cur) cur->text += line + "\n";
  }
  return out;
}

}  // namespace

// Compiles the user invariants of a model (the definitions in m.user_defs
// named by m.invariants[q] - INV_USER) into P; false with a message naming
// the invariant and the construct otherwise.
bool compile_user_invariants(const tlcg_model& m, const HostModel& hm, const std::vector<std::string>& names,
                             UserProg* P, std::string* err) {
  std::memset(P, 0, sizeof *P);
  P->nk = hm.L.nk;
  P->nv = hm.L.nv;
  if (P->nk > UI_MAXSET || P->nv > UI_MAXSET) {
    *err = "KeySet / ValueSet too large for user invariants";
    return false;
  }
  // the packed key / value index is the position in the sorted KeySet / ValueSet (host_model.h)
  for (int i = 0; i < hm.L.nk; ++i) P->keyval[i] = P->keysorted[i] = (int32_t)hm.keyset[(size_t)i];
  for (int i = 0; i < hm.L.nv; ++i) P->valval[i] = P->valsorted[i] = (int32_t)hm.valueset[(size_t)i];
  Compiler c(hm, P);
  for (Def& d : split_defs(m.user_defs ? m.user_defs : "")) c.defs[d.name] = d;
  P->n_user = (int32_t)names.size();
  for (size_t k = 0; k < names.size(); ++k) {
    try {
      c.compile((int)k, names[k]);
    } catch (const CompileError& e) {
      *err = "invariant " + names[k] + " cannot be checked: " + e.what();
      return false;
    }
  }
  return true;
}

// ---------------------------------------------------------------- device code
// The program of every user invariant lowered to straight C++ for the
// run-time specialized kernels (jit.cpp; model.h tlcg_user_eval): one
// function per invariant, the registers as locals, each instruction as the
// interpreter (user_inv.h eval_user_v) executes it, jumps as gotos, the
// KeySet / ValueSet tables as constant expressions.  Under hipRTC the
// layout's constants fold, so a field read is a shift and a mask of the
// engine's own encoding (the view V: a component code, a local key, a word).
namespace {

// x -> t[x] for x in 0..63 (0 past n), as an expression in `x`: arithmetic
// when the table is affine on 0..n-1 with t[0] = 0 (the spec's index 0 is
// NullKey / the null value), else a select chain
std::string table_expr(const int32_t* t, int n, const std::string& x) {
  bool affine = n >= 1 && t[0] == 0;
  long long step = n >= 2 ? (long long)t[1] - t[0] : 1;
  for (int i = 0; i < n && affine; ++i) affine = (long long)t[i] == step * i;
  std::ostringstream o;
  if (affine) {
    o << "((" << x << ") < " << n << " ? " << step << "LL * (" << x << ") : 0LL)";
    return o.str();
  }
  o << "(";
  for (int i = 0; i < n; ++i) o << "(" << x << ") == " << i << " ? " << t[i] << "LL : ";
  o << "0LL)";
  return o.str();
}

// membership of `x` in the ascending t[0..n-1]
std::string member_expr(const int32_t* t, int n, const std::string& x) {
  bool range = n >= 1;
  for (int i = 1; i < n && range; ++i) range = t[i] == t[i - 1] + 1;
  std::ostringstream o;
  if (range) {
    o << "((long long)((" << x << ") >= " << t[0] << "LL && (" << x << ") <= " << t[n - 1] << "LL))";
    return o.str();
  }
  o << "((long long)(false";
  for (int i = 0; i < n; ++i) o << " || (" << x << ") == " << t[i] << "LL";
  o << "))";
  return o.str();
}

}  // namespace

// What user invariant k's program reads of a state (user_fields: component_code.h
// UserField bits; the component constants: UR_LEN, UR_MSGS, UR_LEDB), over the
// instructions reachable from its entry whose result is used.  The lowering
// builds every message record whole (position, key, value), so a program that
// compares ids only still holds dead key / value reads; a backward liveness
// pass over the register program drops those (an instruction is kept when it
// can end the program -- a jump, a return, an error, an overflow check -- or
// when a kept instruction reads its result).
enum UserConstRead : uint32_t { UR_LEN = 1, UR_MSGS = 2, UR_LEDB = 4 };

namespace {

struct InsnRegs {
  uint64_t use = 0, def = 0;
  bool effect = false;  // ends the program or changes control: always kept
};

InsnRegs insn_regs(const UInsn& in) {
  InsnRegs r;
  const uint64_t A = 1ull << in.a, B = 1ull << in.b, C = 1ull << in.c;
  switch (in.op) {
    case U_LDI: case U_LEN: case U_PHASE: case U_P1R: case U_HZ: case U_CTX: case U_CRASH: case U_CURP: case U_CURH:
    case U_CURC:
      r.def = A;
      break;
    case U_MOV: case U_MKEY: case U_MVAL: case U_LEDP: case U_LEDM: case U_NOT: case U_ADDI: case U_POPC: case U_MASK:
    case U_KIN: case U_KAT:
      r.def = A;
      r.use = B;
      break;
    case U_NEG:
      r.def = A;
      r.use = B;
      r.effect = true;  // (the 32-bit overflow error)
      break;
    case U_ADD: case U_SUB: case U_MUL:
      r.def = A;
      r.use = B | C;
      r.effect = true;
      break;
    case U_LFK: case U_DIV: case U_MOD: case U_EQ: case U_NE: case U_LT: case U_LE: case U_AND: case U_OR: case U_BIT:
    case U_NTH:
      r.def = A;
      r.use = B | C;
      break;
    case U_JZ: case U_JNZ: case U_RET:
      r.use = A;
      r.effect = true;
      break;
    default:  // U_JMP, U_ERR, unknown
      r.effect = true;
      break;
  }
  return r;
}

std::vector<int> insn_succ(const UserProg& P, int pc) {
  const UInsn& in = P.ins[pc];
  if (in.op == U_RET || in.op == U_ERR) return {};
  if (in.op == U_JMP) return {in.imm};
  std::vector<int> s{pc + 1};
  if (in.op == U_JZ || in.op == U_JNZ) s.push_back(in.imm);
  return s;
}

// the instructions of P whose effect or result can matter (liveness to a fixpoint)
std::vector<bool> needed_insns(const UserProg& P) {
  const int n = P.n_ins;
  std::vector<uint64_t> live_in((size_t)n + 1, 0);
  std::vector<bool> need((size_t)n, false);
  for (bool changed = true; changed;) {
    changed = false;
    for (int i = n - 1; i >= 0; --i) {
      uint64_t out = 0;
      for (int t : insn_succ(P, i))
        if (t >= 0 && t <= n) out |= live_in[(size_t)t];
      const InsnRegs r = insn_regs(P.ins[i]);
      const bool nd = r.effect || (r.def & out);
      const uint64_t in = nd ? (r.use | (out & ~r.def)) : out;
      if (in != live_in[(size_t)i] || nd != need[(size_t)i]) {
        live_in[(size_t)i] = in;
        need[(size_t)i] = nd;
        changed = true;
      }
    }
  }
  return need;
}

// fields (UserField) and component constants (UserConstRead) read by the
// needed instructions reachable from invariant k's entry
void user_reads(const UserProg& P, const std::vector<bool>& need, int k, uint32_t* fields, uint32_t* consts) {
  const int n = P.n_ins;
  std::vector<bool> seen((size_t)n + 1, false);
  std::vector<int> todo{P.entry[k]};
  uint32_t f = 0, c = 0;
  while (!todo.empty()) {
    const int pc = todo.back();
    todo.pop_back();
    if (pc < 0 || pc >= n || seen[(size_t)pc]) continue;
    seen[(size_t)pc] = true;
    for (int t : insn_succ(P, pc)) todo.push_back(t);
    if (!need[(size_t)pc]) continue;
    switch (P.ins[pc].op) {
      case U_PHASE: f |= UF_PH; break;
      case U_P1R: f |= UF_R; c |= UR_LEN; break;
      case U_HZ: f |= UF_H; c |= UR_LEN; break;
      case U_CTX: f |= UF_X; break;
      case U_CRASH: f |= UF_CR; break;
      case U_CURP: f |= UF_CP; break;
      case U_CURH: f |= UF_CP | UF_CH; c |= UR_LEN; break;
      case U_CURC: f |= UF_CP | UF_CC; break;
      case U_LEDP: f |= UF_LED; break;
      case U_LEDM: f |= UF_LED; c |= UR_LEDB; break;
      case U_LEN: c |= UR_LEN; break;
      case U_MKEY: case U_MVAL: case U_LFK: c |= UR_MSGS; break;
      default: break;
    }
  }
  *fields = f;
  *consts = c;
}

// the class view of the host-made tables: a code and the two constants of a
// class (len, ledbits); any read of `messages` is a read the class does not
// fix (wide), as are UVTab's out-of-range positions
struct UVClass : UVTab<u64> {
  int key(int i) const { wide = true; return UVTab<u64>::key(i); }
  int val(int i) const { wide = true; return UVTab<u64>::val(i); }
};

}  // namespace

uint32_t user_fields(const UserProg& P, int k) {
  uint32_t f = 0, c = 0;
  user_reads(P, needed_insns(P), k, &f, &c);
  return f;
}

uint32_t user_const_reads(const UserProg& P, int k) {
  uint32_t f = 0, c = 0;
  user_reads(P, needed_insns(P), k, &f, &c);
  return c;
}

UserProg user_prune_dead(const UserProg& P) {
  UserProg Q = P;
  const std::vector<bool> need = needed_insns(P);
  for (int i = 0; i < P.n_ins; ++i)
    if (!need[(size_t)i]) Q.ins[i] = UInsn{(uint8_t)U_LDI, P.ins[i].a, 0, 0, 0};  // (its result is never read)
  return Q;
}

u64 user_static_table(const UserProg& P, const Layout& L, int k, uint32_t mask, int len, uint32_t cm) {
  CodeConsts K{};
  K.len = (uint32_t)len;
  K.ledbits = (lkey)(1u | (cm << 1));
  K.msgs = 0;
  if (popcount32(mask) > 5) return ~0ull;  // (more patterns than 64 bits hold: the programs decide)
  u64 t = 0;
  for (int p = 0; p < (1 << popcount32(mask)); ++p) {
    const UVClass v{{{L, K, code_pdep((uint32_t)p, mask)}}};
    const int r = eval_user_v(P, k, v);
    t |= (u64)(v.wide ? 3 : r) << (2 * p);
  }
  return t;
}

std::string user_device_source(const UserProg& P, const Layout& L) {
  std::ostringstream o;
  o << "namespace tlcg {\n";
  const int n = P.n_ins;
  std::vector<bool> target((size_t)n + 1, false);
  for (int k = 0; k < P.n_user; ++k) target[(size_t)P.entry[k]] = true;
  for (int i = 0; i < n; ++i) {
    const UInsn& in = P.ins[i];
    if (in.op == U_JMP || in.op == U_JZ || in.op == U_JNZ) target[(size_t)in.imm] = true;
  }
  int maxreg = 0;
  for (int i = 0; i < n; ++i)
    maxreg = std::max({maxreg, (int)P.ins[i].a + 1, (int)P.ins[i].b + 1, (int)P.ins[i].c + 1});
  maxreg = std::max(maxreg, 1);
  auto R = [](int r) { return "r" + std::to_string(r); };
  for (int k = 0; k < P.n_user; ++k) {
    o << "template <class V>\nTLCG_HD int tlcg_user_inv_" << k << "(const V& v) {\n";
    o << "  long long ";
    for (int r = 0; r < maxreg; ++r) o << R(r) << " = 0" << (r + 1 < maxreg ? ", " : ";\n");
    o << "  int loops = 0;\n  (void)loops;\n";
    o << "  goto L" << P.entry[k] << ";\n";
    for (int i = 0; i < n; ++i) {
      const UInsn& in = P.ins[i];
      if (target[(size_t)i]) o << "L" << i << ":\n";
      const std::string a = R(in.a), b = R(in.b), c = R(in.c);
      auto jump = [&](const std::string& cond) {
        const bool back = in.imm <= i;
        o << "  if (" << cond << ") { ";
        if (back) o << "if (++loops > " << UI_MAXLOOP << ") return EV_ERROR; ";
        o << "goto L" << in.imm << "; }\n";
      };
      const std::string B = b, C = c;
      auto arith = [&](const std::string& e) {
        o << "  { const long long t = " << e << "; if (ui_overflows(t)) return EV_ERROR; " << a << " = t; }\n";
      };
      switch (in.op) {
        case U_LDI: o << "  " << a << " = " << in.imm << "LL;\n"; break;
        case U_MOV: o << "  " << a << " = " << b << ";\n"; break;
        case U_LEN: o << "  " << a << " = v.len();\n"; break;
        case U_MKEY:
          o << "  { const int x = v.key((int)" << b << ") & " << (UI_MAXSET - 1) << "; " << a << " = "
            << table_expr(P.keyval, P.nk, "x") << "; }\n";
          break;
        case U_MVAL:
          o << "  { const int x = v.val((int)" << b << ") & " << (UI_MAXSET - 1) << "; " << a << " = "
            << table_expr(P.valval, P.nv, "x") << "; }\n";
          break;
        case U_PHASE: o << "  " << a << " = " << UV_PHASE0 << "LL + v.phase();\n"; break;
        case U_P1R: o << "  " << a << " = v.p1r();\n"; break;
        case U_HZ: o << "  " << a << " = v.hz();\n"; break;
        case U_CTX: o << "  " << a << " = v.ctx();\n"; break;
        case U_CRASH: o << "  " << a << " = v.crash();\n"; break;
        case U_CURP: o << "  " << a << " = v.curp();\n"; break;
        case U_CURH: o << "  " << a << " = v.curh();\n"; break;
        case U_CURC: o << "  " << a << " = v.curc();\n"; break;
        case U_LEDP: o << "  " << a << " = v.ledp((int)" << b << ");\n"; break;
        case U_LEDM: o << "  " << a << " = (long long)v.ledm((int)" << b << ");\n"; break;
        case U_LFK:
          o << "  { long long best = 0;\n"
            << "    for (int i = 1; i <= (int)" << c << " && i <= v.L.N; ++i) {\n"
            << "      const int x = v.key(i) & " << (UI_MAXSET - 1) << ";\n"
            << "      if (" << table_expr(P.keyval, P.nk, "x") << " == " << b << ") best = i;\n"
            << "    }\n    " << a << " = best; }\n";
          break;
        case U_ADD: arith(B + " + " + C); break;
        case U_SUB: arith(B + " - " + C); break;
        case U_MUL: arith(B + " * " + C); break;
        case U_DIV:
          o << "  { const long long q = " << B << " / " << C << "; " << a << " = (" << B << " % " << C
            << " != 0 && ((" << b << " < 0) != (" << c << " < 0))) ? q - 1 : q; }\n";
          break;
        case U_MOD:
          o << "  { const long long m = " << B << " % " << C << "; " << a << " = m < 0 ? m + " << C << " : m; }\n";
          break;
        case U_NEG: arith("-" + B); break;
        case U_EQ: o << "  " << a << " = " << b << " == " << c << ";\n"; break;
        case U_NE: o << "  " << a << " = " << b << " != " << c << ";\n"; break;
        case U_LT: o << "  " << a << " = " << b << " < " << c << ";\n"; break;
        case U_LE: o << "  " << a << " = " << b << " <= " << c << ";\n"; break;
        case U_NOT: o << "  " << a << " = !" << b << ";\n"; break;
        case U_AND: o << "  " << a << " = " << b << " & " << c << ";\n"; break;
        case U_OR: o << "  " << a << " = " << b << " | " << c << ";\n"; break;
        case U_ADDI: o << "  " << a << " = " << B << " + " << in.imm << "LL;\n"; break;
        case U_BIT:
          o << "  " << a << " = (" << c << " >= 1 && " << c << " <= 63) ? (" << B << " >> (" << c
            << " - 1)) & 1 : 0;\n";
          break;
        case U_POPC: o << "  " << a << " = popcount64((u64)" << b << ");\n"; break;
        case U_NTH: o << "  " << a << " = ui_nth_n(v.L, (u64)" << b << ", " << c << ");\n"; break;
        case U_MASK: o << "  " << a << " = (long long)((1ull << (" << b << " & 63)) - 1);\n"; break;
        case U_KIN:
          o << "  " << a << " = "
            << (in.imm ? member_expr(P.valsorted, P.nv, b) : member_expr(P.keysorted, P.nk, b)) << ";\n";
          break;
        case U_KAT:
          o << "  { const int x = (int)" << b << " & " << (UI_MAXSET - 1) << "; " << a << " = "
            << (in.imm ? table_expr(P.valsorted, P.nv, "x") : table_expr(P.keysorted, P.nk, "x")) << "; }\n";
          break;
        case U_JMP: jump("true"); break;
        case U_JZ: jump("!" + a); break;
        case U_JNZ: jump(a); break;
        case U_ERR: o << "  return EV_ERROR;\n"; break;
        case U_RET: o << "  return " << a << " ? EV_TRUE : EV_FALSE;\n"; break;
        default: o << "  return EV_ERROR;\n"; break;
      }
    }
    if (target[(size_t)n]) o << "L" << n << ":\n";
    o << "  return EV_ERROR;\n}\n";
  }
  o << "template <class V>\nTLCG_HD int tlcg_user_eval(int k, const V& v) {\n  switch (k) {\n";
  for (int k = 0; k < P.n_user; ++k) o << "    case " << k << ": return tlcg_user_inv_" << k << "(v);\n";
  o << "  }\n  return EV_ERROR;\n}\n";
  // the outcome tables (component_code.h code_consts_user): an invariant whose
  // program reads at most UTAB_BITS code bits gets 2 bits per pattern of them
  // in CodeConsts::utab, while its 64 bits last; worked out here for every
  // class (Len, ledger content) when it reads no `messages`, else per
  // component on the device.  TLCG_UTAB=0: none (every state runs the
  // programs; A/B and tests); TLCG_UTAB=dyn: no host-made ones;
  // TLCG_UTAB=slow: every entry 3 (tests: every state takes the kernel's
  // fallback evaluation).
  constexpr int UTAB_BITS = 4;
  const char* ut = std::getenv("TLCG_UTAB");
  const bool tables = !(ut && ut[0] == '0');
  const bool slow = ut && std::string(ut) == "slow";
  const bool statics = !(ut && std::string(ut) == "dyn");
  const std::vector<bool> need = needed_insns(P);
  const UserProg pruned = user_prune_dead(P);  // (the class tables run it: no dead `messages` reads)
  std::vector<int> off((size_t)P.n_user, -1), dyn((size_t)P.n_user, 0);
  std::vector<uint32_t> mask((size_t)P.n_user, 0);
  int used = 0;
  for (int k = 0; k < P.n_user && tables; ++k) {
    uint32_t f = 0, c = 0;
    user_reads(P, need, k, &f, &c);
    const uint32_t m = code_field_mask(L, f);
    const int bits = popcount32(m);
    if (bits > UTAB_BITS || used + (2 << bits) > 64) continue;
    off[(size_t)k] = used;
    mask[(size_t)k] = m;
    dyn[(size_t)k] = ((c & UR_MSGS) || !statics || L.N > 8) && !slow ? 1 : 0;
    used += 2 << bits;
  }
  o << "TLCG_HD int tlcg_user_tab_off(int k) {\n  switch (k) {\n";
  for (int k = 0; k < P.n_user; ++k) o << "    case " << k << ": return " << off[(size_t)k] << ";\n";
  o << "  }\n  return -1;\n}\n";
  o << "TLCG_HD uint32_t tlcg_user_tab_mask(int k) {\n  switch (k) {\n";
  for (int k = 0; k < P.n_user; ++k) o << "    case " << k << ": return " << mask[(size_t)k] << "u;\n";
  o << "  }\n  return 0u;\n}\n";
  o << "TLCG_HD int tlcg_user_tab_dyn(int k) {\n  switch (k) {\n";
  for (int k = 0; k < P.n_user; ++k) o << "    case " << k << ": return " << dyn[(size_t)k] << ";\n";
  o << "  }\n  return 0;\n}\n";
  // the host-made tables: class (len, cm) at index len << N | cm, cm the
  // ledger content's position mask (CodeConsts ledbits >> 1); a class past
  // them (none is reachable: Len(messages) <= N) reads all 3s
  u64 smask = 0;
  for (int k = 0; k < P.n_user; ++k)
    if (off[(size_t)k] >= 0 && !dyn[(size_t)k])
      smask |= (((2 << popcount32(mask[(size_t)k])) >= 64 ? ~0ull : (1ull << (2 << popcount32(mask[(size_t)k]))) - 1)
               << off[(size_t)k]);
  if (!smask) {
    o << "TLCG_HD u64 tlcg_user_tab_static(const CodeConsts&) { return 0; }\n";
  } else if (slow) {
    o << "TLCG_HD u64 tlcg_user_tab_static(const CodeConsts&) { return " << smask << "ull; }\n";
  } else {
    const int ncls = (L.N + 1) << L.N;
    o << "__constant__ const u64 kUTabStatic[" << ncls << "] = {";
    for (int len = 0; len <= L.N; ++len)
      for (uint32_t cm = 0; cm < (1u << L.N); ++cm) {
        u64 t = 0;
        for (int k = 0; k < P.n_user; ++k)
          if (off[(size_t)k] >= 0 && !dyn[(size_t)k])
            t |= user_static_table(pruned, L, k, mask[(size_t)k], len, cm) << off[(size_t)k];
        o << t << "ull" << (len == L.N && cm + 1 == (1u << L.N) ? "" : ", ");
      }
    o << "};\n";
    o << "TLCG_HD u64 tlcg_user_tab_static(const CodeConsts& K) {\n"
      << "  const uint32_t cm = (uint32_t)(K.ledbits >> 1);\n"
      << "  return K.len <= " << L.N << "u && cm < " << (1u << L.N) << "u ? kUTabStatic[(K.len << " << L.N
      << ") | cm] : " << smask << "ull;\n}\n";
  }
  o << "}  // namespace tlcg\n";
  return o.str();
}

// the names of the definitions in a user_defs text, in order
std::vector<std::string> user_def_names(const char* text) {
  std::vector<std::string> out;
  for (const Def& d : split_defs(text ? text : "")) out.push_back(d.name);
  return out;
}

}  // namespace tlcg
