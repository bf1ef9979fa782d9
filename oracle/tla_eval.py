"""oracle/tla_eval.py -- TEST INFRASTRUCTURE ONLY: evaluator of user invariants
(TLA+ state predicates added to compaction.tla) over the Python oracle's values.

Written independently of the product's compiler (pulsar-tlaplus_amd/csrc/
user_inv.cpp): it parses the definition text itself and evaluates the
expression tree directly on TLC-like Python values -- nothing is lowered or
typed ahead of time.  oracle_py.Model uses it for invariants named in
`user_defs`; the tests compare it with the product on every reachable state
and on whole runs (tests/test_user_inv*.py).  Never imported by the product.

Values (TLC's):
  integers          int (never bool)
  booleans          bool
  model values      MV("Nil"), MV("Compactor_In_PhaseOne"), ...  (equal only to themselves)
  records           Rec (sorted (field, value) pairs)
  sequences         tuple (a function with domain 1..n)
  functions         Fcn (domain frozenset -> value); one with domain 1..n is a tuple
  sets              frozenset
Evaluation errors raise EvalError, as TLC would stop with one.
"""
from __future__ import annotations

import re

PHASES = ("Compactor_In_PhaseOne", "Compactor_In_PhaseTwoWrite", "Compactor_In_PhaseTwoUpdateContext",
          "Compactor_In_PhaseTwoUpdateHorizon", "Compactor_In_PhaseTwoPersistCusror",
          "Compactor_In_PhaseTwoDeleteLedger")  # compaction.tla:39-44


class EvalError(Exception):
    pass


class Unsupported(Exception):
    pass


class MV:
    __slots__ = ("name",)

    def __init__(self, name):
        self.name = name

    def __eq__(self, o):
        return isinstance(o, MV) and o.name == self.name

    def __hash__(self):
        return hash(("MV", self.name))

    def __repr__(self):
        return self.name


NIL = MV("Nil")


class Rec:
    __slots__ = ("f",)

    def __init__(self, **kw):
        self.f = tuple(sorted(kw.items()))

    def get(self, k):
        for a, b in self.f:
            if a == k:
                return b
        raise EvalError(f"record has no field {k}")

    def fields(self):
        return {a for a, _ in self.f}

    def __eq__(self, o):
        return isinstance(o, Rec) and o.f == self.f

    def __hash__(self):
        return hash(("Rec", self.f))


class Fcn:
    __slots__ = ("m",)

    def __init__(self, m):
        self.m = dict(m)

    def __eq__(self, o):
        return isinstance(o, Fcn) and o.m == self.m

    def __hash__(self):
        return hash(("Fcn", tuple(sorted(self.m.items(), key=repr))))


class LazyFcn:
    r"""[x \in S |-> e] as TLC keeps it (FcnLambdaValue): f[a] evaluates e at a
    only; equality, DOMAIN, Len and the like build the whole function"""
    __slots__ = ("dom", "var", "body", "cx", "ev")

    def __init__(self, dom, var, body, cx, ev):
        self.dom, self.var, self.body, self.cx, self.ev = dom, var, body, cx, ev

    def at(self, a):
        if not any(kind(a) == kind(x) and teq(a, x) for x in self.dom):
            raise EvalError("argument out of the function's domain")
        return self.ev.ev(self.body, self.ev.bind(self.cx, self.var, a))

    def force(self):
        return Fcn({x: self.at(x) for x in self.ev.sorted_set(self.dom)})


def norm(v):
    """a function with domain 1..n is the sequence of its values"""
    if isinstance(v, LazyFcn):
        v = v.force()
    if isinstance(v, Fcn):
        ks = list(v.m)
        if all(type(k) is int for k in ks) and sorted(ks) == list(range(1, len(ks) + 1)):
            return tuple(v.m[i] for i in range(1, len(ks) + 1))
    return v


def kind(v):
    v = norm(v)
    if isinstance(v, bool):
        return "bool"
    if isinstance(v, int):
        return "int"
    if isinstance(v, MV):
        return "mv"
    if isinstance(v, Rec):
        return "rec"
    if isinstance(v, (tuple, Fcn)):
        return "fcn"
    if isinstance(v, frozenset):
        return "set"
    return type(v).__name__


def teq(a, b):
    """TLC equality: a model value differs from every other value; others must be comparable"""
    a, b = norm(a), norm(b)
    ka, kb = kind(a), kind(b)
    if ka == "mv" or kb == "mv":
        return ka == kb and a == b
    if ka != kb:
        raise EvalError(f"cannot compare {ka} with {kb}")
    if ka == "rec":
        if a.fields() != b.fields():
            return False
        return all(teq(a.get(k), b.get(k)) for k in a.fields())
    if ka == "fcn":
        if isinstance(a, tuple) and isinstance(b, tuple):
            return len(a) == len(b) and all(teq(x, y) for x, y in zip(a, b))
        return a == b
    if ka == "set":
        return len(a) == len(b) and all(any(teq(x, y) for y in b) for x in a)
    return a == b


# ---------------------------------------------------------------- lexer / parser
_TOK = re.compile(r"""
   (?P<ws>[ \t\r]+) | (?P<nl>\n) | (?P<cmt>\\\*[^\n]*)
 | (?P<num>\d+) | (?P<id>[A-Za-z_][A-Za-z0-9_]*) | (?P<str>"[^"]*")
 | (?P<bs>\\[A-Za-z]+)
 | (?P<op><=>|\|->|==|/\\|\\/|=>|/=|<=|=<|>=|\.\.|<<|>>|->|\[\]|[=\#<>+\-*%()\[\]{},:.~'\\])
""", re.X)


def tokenize(text, line0=1):
    # nested (* *) comments first
    out, i, depth = [], 0, 0
    buf = []
    while i < len(text):
        if text.startswith("(*", i):
            depth += 1
            buf.append("  ")
            i += 2
        elif depth and text.startswith("*)", i):
            depth -= 1
            buf.append("  ")
            i += 2
        elif depth:
            buf.append("\n" if text[i] == "\n" else " ")
            i += 1
        else:
            buf.append(text[i])
            i += 1
    text = "".join(buf)
    line, col, pos = line0, 1, 0
    while pos < len(text):
        m = _TOK.match(text, pos)
        if not m:
            raise Unsupported(f"bad character {text[pos]!r}")
        k = m.lastgroup
        s = m.group()
        if k == "nl":
            line, col = line + 1, 1
        elif k not in ("ws", "cmt"):
            out.append((k, s, line, col))
        if k != "nl":
            col += len(s)
        pos = m.end()
    out.append(("end", "", line, 0))
    return out


ALIAS = {"\\land": "/\\", "\\lor": "\\/", "\\equiv": "<=>", "=<": "<=", "\\leq": "<=", "\\geq": ">=", "/=": "#",
         "\\union": "\\cup", "\\intersect": "\\cap", "\\lnot": "~", "\\neg": "~", "\\forall": "\\A",
         "\\exists": "\\E"}
BIN = {"=>": (1, "r"), "<=>": (2, "n"), "/\\": (3, "l"), "\\/": (3, "l"), "=": (5, "n"), "#": (5, "n"),
       "<": (5, "n"), ">": (5, "n"), "<=": (5, "n"), ">=": (5, "n"), "\\in": (5, "n"), "\\notin": (5, "n"),
       "\\subseteq": (5, "n"), "\\cup": (8, "l"), "\\cap": (8, "l"), "\\": (8, "l"), "..": (9, "n"),
       "+": (10, "l"), "-": (10, "l"), "%": (10, "n"), "*": (13, "l"), "\\div": (13, "l")}


class Parser:
    def __init__(self, toks):
        self.t = [(k, ALIAS.get(s, s), l, c) for k, s, l, c in toks]
        self.p = 0
        self.fences = []

    def peek(self, k=0, fenced=True):
        tok = self.t[min(self.p + k, len(self.t) - 1)]
        if fenced and k == 0 and self.fences and tok[0] != "end" and tok[3] <= self.fences[-1]:
            return ("end", "", tok[2], tok[3])
        return tok

    def at(self, s):
        k, v, _, _ = self.peek()
        return k in ("op", "bs", "id") and v == s

    def eat(self, s):
        if not self.at(s):
            raise Unsupported(f"expected {s!r} at line {self.peek()[2]}, found {self.peek()[1]!r}")
        self.p += 1

    def ident(self):
        k, v, _, _ = self.peek()
        if k != "id":
            raise Unsupported(f"expected an identifier, found {v!r}")
        self.p += 1
        return v

    def expr(self, minp=0):
        lhs = self.unary()
        while True:
            k, v, _, _ = self.peek()
            if k not in ("op", "bs") or v not in BIN or BIN[v][0] < minp:
                return lhs
            prec, assoc = BIN[v]
            self.p += 1
            rhs = self.expr(prec + 1)
            lhs = ("bin", v, lhs, rhs)

    def unary(self):
        if self.at("~"):
            self.p += 1
            return ("not", self.expr(4))
        if self.at("-"):
            self.p += 1
            return ("neg", self.expr(12))
        return self.post(self.primary())

    def post(self, e):
        while True:
            if self.at("["):
                self.p += 1
                a = self.expr()
                self.eat("]")
                e = ("app", e, a)
            elif self.at(".") and self.peek(1)[0] == "id":
                self.p += 1
                e = ("field", e, self.ident())
            else:
                return e

    def bounds(self):
        out = []
        while True:
            names = [self.ident()]
            while self.at(","):
                self.p += 1
                names.append(self.ident())
            self.eat("\\in")
            s = self.expr(6)
            out += [(n, s) for n in names]
            if not self.at(","):
                return out
            self.p += 1

    def primary(self):
        k, v, line, col = self.peek()
        if k == "end":
            raise Unsupported("unexpected end")
        if k == "num":
            self.p += 1
            return ("num", int(v))
        if k in ("op", "bs") and v in ("/\\", "\\/"):
            items = []
            while True:
                self.p += 1
                self.fences.append(col)
                items.append(self.expr())
                self.fences.pop()
                nk, nv, _, nc = self.peek(fenced=False)
                if not (nv == v and nc == col and (not self.fences or nc > self.fences[-1])):
                    break
            return ("junct", v, items)
        if self.at("("):
            self.p += 1
            self.fences.append(-1)
            e = self.expr()
            self.fences.pop()
            self.eat(")")
            return e
        if k == "bs" and v in ("\\A", "\\E"):
            self.p += 1
            b = self.bounds()
            self.eat(":")
            return ("quant", v, b, self.expr())
        if k == "id":
            if v in ("TRUE", "FALSE"):
                self.p += 1
                return ("bool", v == "TRUE")
            if v == "IF":
                self.p += 1
                c = self.expr()
                self.eat("THEN")
                a = self.expr()
                self.eat("ELSE")
                return ("if", c, a, self.expr())
            if v == "CASE":
                self.p += 1
                arms, other = [], None
                while True:
                    if self.at("OTHER"):
                        self.p += 1
                        self.eat("->")
                        other = self.expr()
                        break
                    g = self.expr()
                    self.eat("->")
                    arms.append((g, self.expr()))
                    if not self.at("[]"):
                        break
                    self.p += 1
                return ("case", arms, other)
            if v == "LET":
                self.p += 1
                defs = []
                while not self.at("IN"):
                    n = self.ident()
                    ps = []
                    if self.at("("):
                        self.p += 1
                        ps.append(self.ident())
                        while self.at(","):
                            self.p += 1
                            ps.append(self.ident())
                        self.eat(")")
                    self.eat("==")
                    self.fences.append(-1)
                    defs.append((n, ps, self.expr()))
                    self.fences.pop()
                self.eat("IN")
                return ("let", defs, self.expr())
            if v == "CHOOSE":
                self.p += 1
                n = self.ident()
                self.eat("\\in")
                s = self.expr(6)
                self.eat(":")
                return ("choose", n, s, self.expr())
            if v == "DOMAIN":
                self.p += 1
                return ("domain", self.post(self.primary()))
            self.p += 1
            if self.at("("):
                self.p += 1
                self.fences.append(-1)
                args = [self.expr()]
                while self.at(","):
                    self.p += 1
                    args.append(self.expr())
                self.fences.pop()
                self.eat(")")
                return ("call", v, args)
            return ("name", v)
        if self.at("{"):
            self.p += 1
            self.fences.append(-1)
            if self.at("}"):
                e = ("setenum", [])
            elif self.peek()[0] == "id" and self.peek(1)[1] == "\\in" and self._filter_ahead():
                n = self.ident()
                self.eat("\\in")
                s = self.expr(6)
                self.eat(":")
                e = ("filter", n, s, self.expr())
            else:
                first = self.expr()
                if self.at(":"):
                    self.p += 1
                    e = ("setmap", first, self.bounds())
                else:
                    items = [first]
                    while self.at(","):
                        self.p += 1
                        items.append(self.expr())
                    e = ("setenum", items)
            self.fences.pop()
            self.eat("}")
            return e
        if self.at("<<"):
            self.p += 1
            items = []
            if not self.at(">>"):
                items.append(self.expr())
                while self.at(","):
                    self.p += 1
                    items.append(self.expr())
            self.eat(">>")
            return ("tuple", items)
        if self.at("["):
            self.p += 1
            self.fences.append(-1)
            if self.peek()[0] == "id" and self.peek(1)[1] == "\\in":
                n = self.ident()
                self.eat("\\in")
                s = self.expr(6)
                self.eat("|->")
                e = ("fctor", n, s, self.expr())
            elif self.peek()[0] == "id" and self.peek(1)[1] in ("|->", ":"):
                sep = self.peek(1)[1]
                fs = []
                while True:
                    f = self.ident()
                    self.eat(sep)
                    fs.append((f, self.expr()))
                    if not self.at(","):
                        break
                    self.p += 1
                e = ("record" if sep == "|->" else "recset", fs)
            else:
                raise Unsupported("unsupported [...] form")
            self.fences.pop()
            self.eat("]")
            return e
        raise Unsupported(f"unexpected {v!r} at line {line}")

    def _filter_ahead(self):
        depth = 0
        for k, v, _, _ in self.t[self.p + 2:]:
            if k == "end":
                return False
            if v in ("(", "[", "{", "<<"):
                depth += 1
            elif v in (")", "]", ">>"):
                depth -= 1
            elif v == "}":
                if depth == 0:
                    return False
                depth -= 1
            elif v == ":" and depth == 0:
                return True
            elif v == "," and depth == 0:
                return False
        return False


# ---------------------------------------------------------------- evaluator
class Evaluator:
    """Evaluates user definitions (name -> (params, body text)) on one oracle state"""

    def __init__(self, model, user_defs):
        self.model = model
        self.defs = {}
        for head, body in user_defs.items():
            name, _, rest = head.partition("(")
            params = [p.strip() for p in rest.rstrip(")").split(",") if p.strip()]
            self.defs[name.strip()] = (params, body)
        self.parsed = {}

    def body(self, name):
        if name not in self.parsed:
            params, text = self.defs[name]
            p = Parser(tokenize(text))
            e = p.expr()
            if p.peek()[0] != "end":
                raise Unsupported(f"trailing text in {name}")
            self.parsed[name] = (params, e)
        return self.parsed[name]

    def state_env(self, s):
        msgs, led, cur, ph, p1r, hz, ctx, crash, cons = s
        m = self.model
        msg = lambda t: Rec(id=t[0], key=t[1], value=t[2])  # noqa: E731
        v = {
            "messages": tuple(msg(t) for t in msgs),
            "compactedLedgers": tuple(NIL if l is None else tuple(msg(t) for t in l) for l in led),
            "cursor": NIL if cur is None else Rec(compactionHorizon=cur[0], compactedTopicContext=cur[1]),
            "compactorState": MV(PHASES[ph]),
            "phaseOneResult": NIL if p1r is None else Rec(readPosition=p1r[0], latestForKey=Fcn(dict(p1r[1]))),
            "compactionHorizon": hz, "compactedTopicContext": ctx, "crashTimes": crash, "consumeTimes": cons,
            "MessageSentLimit": m.N, "CompactionTimesLimit": m.C, "MaxCrashTimes": m.K, "ConsumeTimesLimit": m.ctl,
            "ModelConsumer": m.consumer, "ModelProducer": m.producer, "RetainNullKey": m.retain,
            "KeySpace": frozenset(k for k in m.keyset if k != 0),
            "ValueSpace": frozenset(x for x in m.valueset if x != 0),
            "Nil": NIL, "BOOLEAN": frozenset({False, True}),
        }
        for ph_name in PHASES:
            v[ph_name] = MV(ph_name)
        return v

    def holds(self, name, s):
        """True / False; raises EvalError"""
        params, e = self.body(name)
        if getattr(self, "_last", (None,))[0] is not s:  # (the state's values, built once per state)
            self._last = (s, self.state_env(s))
        r = self.ev(e, dict(state=self._last[1], env={}))
        if not isinstance(r, bool):
            raise EvalError("invariant is not a boolean")
        return r

    # ---- expressions
    def ev(self, e, cx):
        op = e[0]
        if op == "num":
            return e[1]
        if op == "bool":
            return e[1]
        if op == "name":
            return self.name(e[1], [], cx)
        if op == "call":
            return self.name(e[1], e[2], cx)
        if op == "not":
            return not self.boolean(e[1], cx)
        if op == "neg":
            return -self.integer(e[1], cx)
        if op == "junct":
            if e[1] == "/\\":
                return all(self.boolean(x, cx) for x in e[2])
            return any(self.boolean(x, cx) for x in e[2])
        if op == "if":
            return self.ev(e[2], cx) if self.boolean(e[1], cx) else self.ev(e[3], cx)
        if op == "case":
            for g, x in e[1]:
                if self.boolean(g, cx):
                    return self.ev(x, cx)
            if e[2] is None:
                raise EvalError("no CASE arm applies")
            return self.ev(e[2], cx)
        if op == "let":
            env = dict(cx["env"])
            for n, ps, body in e[1]:
                env[n] = ("def", ps, body, None)
            cx2 = dict(cx, env=env)
            for n in list(env):  # LET definitions see their own scope
                if env[n][0] == "def" and env[n][3] is None:
                    env[n] = ("def", env[n][1], env[n][2], cx2)
            return self.ev(e[2], cx2)
        if op == "quant":
            return self.quant(e[1], e[2], e[3], cx)
        if op == "choose":
            s = self.setv(e[2], cx)
            good = [x for x in s if self.boolean(e[3], self.bind(cx, e[1], x))]
            if not good:
                raise EvalError("CHOOSE: no element")
            if not all(type(x) is int for x in good):
                raise Unsupported("CHOOSE over non-integers")
            return min(good)
        if op == "setenum":
            out = []
            for x in e[1]:
                v = self.ev(x, cx)
                if not any(teq(v, y) for y in out):
                    out.append(v)
            return frozenset(norm(v) for v in out)
        if op == "filter":
            s = self.setv(e[2], cx)
            return frozenset(x for x in s if self.boolean(e[3], self.bind(cx, e[1], x)))
        if op == "setmap":
            out = []

            def rec(i, c):
                if i == len(e[2]):
                    out.append(norm(self.ev(e[1], c)))
                    return
                n, s = e[2][i]
                for x in self.sorted_set(self.setv(s, c)):
                    rec(i + 1, self.bind(c, n, x))
            rec(0, cx)
            return frozenset(out)
        if op == "tuple":
            return tuple(self.ev(x, cx) for x in e[1])
        if op == "record":
            return Rec(**{f: self.ev(x, cx) for f, x in e[1]})
        if op == "recset":
            return ("recset", [(f, self.setv(x, cx)) for f, x in e[1]])
        if op == "fctor":
            return LazyFcn(self.setv(e[2], cx), e[1], e[3], cx, self)
        if op == "domain":
            f = norm(self.ev(e[1], cx))
            if isinstance(f, tuple):
                return frozenset(range(1, len(f) + 1))
            if isinstance(f, Fcn):
                return frozenset(f.m)
            raise EvalError("DOMAIN of a non-function")
        if op == "app":
            f = self.ev(e[1], cx)
            x = self.ev(e[2], cx)
            if isinstance(f, LazyFcn):
                return f.at(x)
            f = norm(f)
            if isinstance(f, tuple):
                if type(x) is not int or not 1 <= x <= len(f):
                    raise EvalError("index out of the sequence's domain")
                return f[x - 1]
            if isinstance(f, Fcn):
                for k, v in f.m.items():
                    if kind(k) == kind(x) and teq(k, x):
                        return v
                raise EvalError("argument out of the function's domain")
            raise EvalError("application of a non-function")
        if op == "field":
            r = self.ev(e[1], cx)
            if not isinstance(r, Rec):
                raise EvalError("field of a non-record")
            return r.get(e[2])
        if op == "bin":
            return self.binary(e[1], e[2], e[3], cx)
        raise Unsupported(op)

    def name(self, n, args, cx):
        env = cx["env"]
        if n in env:
            b = env[n]
            if b[0] == "val":
                return b[1]
            _, ps, body, dcx = b
            return self.apply_def(ps, body, dcx, args, cx)
        if n in self.defs:
            ps, body = self.body(n)
            return self.apply_def(ps, body, dict(state=cx["state"], env={}), args, cx)
        if n == "Len":
            s = norm(self.ev(args[0], cx))
            if not isinstance(s, tuple):
                raise EvalError("Len of a non-sequence")
            return len(s)
        if n == "Cardinality":
            return len(self.setv(args[0], cx))
        if n == "Head":
            s = norm(self.ev(args[0], cx))
            if not isinstance(s, tuple) or not s:
                raise EvalError("Head of an empty sequence")
            return s[0]
        if args:
            raise Unsupported(f"operator {n}")
        if n in cx["state"]:
            return cx["state"][n]
        if n in ("Nat", "Int"):
            return ("inf", n)
        raise Unsupported(f"unknown name {n}")

    def apply_def(self, ps, body, dcx, args, cx):
        if len(ps) != len(args):
            raise Unsupported("arity")
        env = dict(dcx["env"])
        for p, a in zip(ps, args):
            env[p] = ("def", [], a, cx)  # by name, in the caller's context
        return self.ev(body, dict(dcx, env=env))

    def bind(self, cx, n, v):
        env = dict(cx["env"])
        env[n] = ("val", v)
        return dict(cx, env=env)

    def boolean(self, e, cx):
        v = self.ev(e, cx)
        if not isinstance(v, bool):
            raise EvalError("not a boolean")
        return v

    def integer(self, e, cx):
        v = self.ev(e, cx)
        if type(v) is not int:
            raise EvalError("not an integer")
        return v

    def setv(self, e, cx):
        v = self.ev(e, cx)
        if isinstance(v, frozenset):
            return v
        raise EvalError("not an enumerable set") if not isinstance(v, tuple) else EvalError("a sequence is not a set")

    @staticmethod
    def sorted_set(s):
        return sorted(s, key=lambda x: (kind(x), x if type(x) is int else repr(x)))

    def member(self, x, se, cx):
        s = self.ev(se, cx)
        if isinstance(s, tuple) and s and s[0] == "inf":
            return type(x) is int and (s[1] == "Int" or x >= 0)
        if isinstance(s, tuple) and s and s[0] == "recset":
            if not isinstance(x, Rec) or x.fields() != {f for f, _ in s[1]}:
                return False
            return all(any(kind(y) == kind(x.get(f)) and teq(y, x.get(f)) for y in vs) for f, vs in s[1])
        if not isinstance(s, frozenset):
            raise EvalError("\\in a non-set")
        return any((kind(y) == kind(x) or "mv" in (kind(x), kind(y))) and teq(y, x) for y in s)

    def quant(self, q, bounds, body, cx):
        def rec(i, c):
            if i == len(bounds):
                return self.boolean(body, c)
            n, se = bounds[i]
            s = self.setv(se, c)
            it = (rec(i + 1, self.bind(c, n, x)) for x in self.sorted_set(s))
            return all(it) if q == "\\A" else any(it)
        return rec(0, cx)

    def binary(self, op, a, b, cx):
        if op == "/\\":
            return self.boolean(a, cx) and self.boolean(b, cx)
        if op == "\\/":
            return self.boolean(a, cx) or self.boolean(b, cx)
        if op == "=>":
            return (not self.boolean(a, cx)) or self.boolean(b, cx)
        if op == "<=>":
            return self.boolean(a, cx) == self.boolean(b, cx)
        if op in ("=", "#"):
            r = teq(self.ev(a, cx), self.ev(b, cx))
            return r if op == "=" else not r
        if op in ("\\in", "\\notin"):
            x = norm(self.ev(a, cx))
            r = self.member(x, b, cx)
            return r if op == "\\in" else not r
        if op == "\\subseteq":
            A, B = self.setv(a, cx), self.setv(b, cx)
            return all(any(teq(x, y) for y in B) for x in A)
        if op in ("\\cup", "\\cap", "\\"):
            A, B = self.setv(a, cx), self.setv(b, cx)
            inb = lambda x: any(kind(x) == kind(y) and teq(x, y) for y in B)  # noqa: E731
            if op == "\\cup":
                return A | frozenset(y for y in B if not any(kind(x) == kind(y) and teq(x, y) for x in A))
            if op == "\\cap":
                return frozenset(x for x in A if inb(x))
            return frozenset(x for x in A if not inb(x))
        if op == "..":
            lo, hi = self.integer(a, cx), self.integer(b, cx)
            return frozenset(range(lo, hi + 1))
        x, y = self.integer(a, cx), self.integer(b, cx)
        if op == "+":
            return x + y
        if op == "-":
            return x - y
        if op == "*":
            return x * y
        if op == "\\div":
            if y == 0:
                raise EvalError("division by zero")
            return x // y
        if op == "%":
            if y <= 0:
                raise EvalError("% by a non-positive number")
            return x % y
        return {"<": x < y, "<=": x <= y, ">": x > y, ">=": x >= y}[op]
