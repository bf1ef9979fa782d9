"""oracle/oracle_py.py -- TEST INFRASTRUCTURE ONLY (second, independent oracle).

A pure-Python restatement of compaction.tla's Init/Next/invariants over
immutable Python values (tuples / frozensets / None for the model value Nil),
written separately from oracle/tlc_oracle.c so the two restatements can
cross-check each other on small constants.  Pure-Python loops: use it only on
state spaces of at most a few 1e5 states.  Never imported by the product.

Value model (TLC values):
  message          (id, key, value)                      ConstructMessage, compaction.tla:80-81
  messages         tuple of messages                      compaction.tla:57
  compactedLedgers tuple, index i-1 holds ledger i: None (Nil) or tuple of messages
  cursor           None or (compactionHorizon, compactedTopicContext)   compaction.tla:150
  phaseOneResult   None or (readPosition, latestForKey as sorted tuple of (key, index))  :97-98
Counting conventions follow TLC with one worker (see tlc_oracle.c header).
"""
from __future__ import annotations

from collections import deque

P1, W, UC, UH, PER, DEL = range(6)  # compaction.tla:39-44
ACTIONS = ("Producer", "CompactorPhaseOne", "CompactorPhaseTwoWrite",
           "CompactorPhaseTwoUpdateContext", "CompactorPhaseTwoUpdateHorizon",
           "CompactorPhaseTwoPersistCusror", "CompactorPhaseTwoDeleteLedger",
           "BrokerCrash", "Consumer", "Terminating")  # Next order, compaction.tla:216-231


class EvalError(Exception):
    pass


class Model:
    def __init__(self, N=3, C=3, K=1, keys=(1, 2), values=(1, 2), retain=True,
                 producer=False, consumer=False, ctl=2,
                 invariants=("TypeSafe", "CompactionHorizonCorrectness"), deadlock=True, user_defs=None):
        self.N, self.C, self.K, self.ctl = N, C, K, ctl
        self.keyset = sorted(set(keys) | {0})      # KeySet, compaction.tla:49
        self.valueset = sorted(set(values) | {0})  # ValueSet, compaction.tla:50
        self.retain, self.producer, self.consumer = retain, producer, consumer
        self.invariants, self.deadlock = tuple(invariants), deadlock
        # invariants the user added to the module (BASELINE config 5): their own
        # parser/evaluator, oracle/tla_eval.py (test infrastructure)
        self.user = None
        if user_defs:
            from tla_eval import Evaluator
            self.user = Evaluator(self, user_defs)

    # state = (messages, ledgers, cursor, phase, p1r, horizon, context, crash, consume)
    def inits(self):
        base = (None,) * self.C
        if self.producer:
            yield ((), base, None, P1, None, 0, 0, 0, 0)
            return
        per = [(k, v) for v in self.valueset for k in self.keyset]  # key fastest
        n = len(per)
        for idx in range(n ** self.N):
            msgs, r = [], idx
            for i in range(self.N):
                k, v = per[r % n]
                r //= n
                msgs.append((i + 1, k, v))
            yield (tuple(msgs), base, None, P1, None, 0, 0, 0, 0)

    def max_ledger(self, led):  # MaxCompactedLedgerId, compaction.tla:103-106
        ids = [i + 1 for i, l in enumerate(led) if l is not None]
        return max(ids) if ids else 0

    def successors(self, s):
        """Yield (action_index, successor) in Next order; raise EvalError."""
        msgs, led, cur, ph, p1r, hz, ctx, crash, cons = s
        if self.producer and len(msgs) < self.N:  # Producer, :83-87
            for k in self.keyset:
                for v in self.valueset:
                    yield 0, (msgs + ((len(msgs) + 1, k, v),), led, cur, ph, p1r, hz, ctx, crash, cons)
        if ph == P1 and p1r is None and len(msgs) > 0:  # CompactorPhaseOne, :93-100
            latest = tuple((k, max(i + 1 for i, m in enumerate(msgs) if m[1] == k))
                           for k in sorted({m[1] for m in msgs} - {0}))
            yield 1, (msgs, led, cur, W, (len(msgs), latest), hz, ctx, crash, cons)
        if p1r is not None and ph == W:  # CompactorPhaseTwoWrite, :121-132
            nid = self.max_ledger(led) + 1
            if 1 <= nid <= self.C:
                rp, latest = p1r
                lf = dict(latest)
                out = []
                for i in range(1, rp + 1):  # CompactMessages, :107-119
                    m = msgs[i - 1]
                    if m[1] == 0:
                        keep = self.retain
                    else:
                        if m[1] not in lf:
                            raise EvalError("latestForKey domain")
                        keep = (i == lf[m[1]])
                    if keep:
                        out.append(m)
                nl = list(led)
                nl[nid - 1] = tuple(out)
                yield 2, (msgs, tuple(nl), cur, UC, p1r, hz, ctx, crash, cons)
        if ph == UC:  # :135-139
            yield 3, (msgs, led, cur, UH, p1r, hz, self.max_ledger(led), crash, cons)
        if ph == UH:  # :141-145
            if p1r is None:
                raise EvalError("readPosition of Nil")
            yield 4, (msgs, led, cur, PER, p1r, p1r[0], ctx, crash, cons)
        if ph == PER:  # :147-151
            yield 5, (msgs, led, (hz, ctx), DEL, p1r, hz, ctx, crash, cons)
        if ph == DEL:  # :153-165
            mx = self.max_ledger(led)
            nl = led
            if mx != 1:
                old = mx - 1
                if not 1 <= old <= self.C:
                    raise EvalError("ledger index")
                if led[old - 1] is not None:
                    l2 = list(led)
                    l2[old - 1] = None
                    nl = tuple(l2)
            yield 6, (msgs, nl, cur, P1, None, hz, ctx, crash, cons)
        yield from self.tail_actions(s)

    def tail_actions(self, s):
        """The disjuncts after the compactor's (:227-230), which never fail."""
        msgs, led, cur, ph, p1r, hz, ctx, crash, cons = s
        if crash < self.K:  # BrokerCrash, :169-182
            h, c = cur if cur is not None else (0, 0)
            yield 7, (msgs, led, cur, P1, None, h, c, crash + 1, cons)
        if self.consumer:  # Consumer, :185-186
            yield 8, s
        if (len(msgs) == self.N and ph == W and self.max_ledger(led) == self.C
                and (not self.consumer or cons == self.ctl)):  # Terminating, :205-214
            yield 9, s

    # ---- TLC value syntax of a state (variables in declaration order, compaction.tla:57-70) ----
    @staticmethod
    def render(s):
        msgs, led, cur, ph, p1r, hz, ctx, crash, cons = s
        names = ("Compactor_In_PhaseOne", "Compactor_In_PhaseTwoWrite", "Compactor_In_PhaseTwoUpdateContext",
                 "Compactor_In_PhaseTwoUpdateHorizon", "Compactor_In_PhaseTwoPersistCusror",
                 "Compactor_In_PhaseTwoDeleteLedger")

        def seq(ms):
            return "<<" + ", ".join(f"[id |-> {i}, key |-> {k}, value |-> {v}]" for i, k, v in ms) + ">>"

        if p1r is None:
            p1 = "Nil"
        else:
            dom = [k for k, _ in p1r[1]]
            f = ("<<" + ", ".join(str(v) for _, v in p1r[1]) + ">>" if dom == list(range(1, len(dom) + 1))
                 else "(" + " @@ ".join(f"{k} :> {v}" for k, v in p1r[1]) + ")")
            p1 = f"[latestForKey |-> {f}, readPosition |-> {p1r[0]}]"
        return "\n".join([
            "/\\ messages = " + seq(msgs),
            "/\\ compactedLedgers = <<" + ", ".join("Nil" if l is None else seq(l) for l in led) + ">>",
            "/\\ cursor = " + ("Nil" if cur is None else
                               f"[compactedTopicContext |-> {cur[1]}, compactionHorizon |-> {cur[0]}]"),
            "/\\ compactorState = " + names[ph],
            "/\\ phaseOneResult = " + p1,
            f"/\\ compactionHorizon = {hz}", f"/\\ compactedTopicContext = {ctx}",
            f"/\\ crashTimes = {crash}", f"/\\ consumeTimes = {cons}"])

    # ---- invariants ----
    def ledger_at_ctx(self, s):
        led, ctx = s[1], s[6]
        if not 1 <= ctx <= self.C or led[ctx - 1] is None:
            raise EvalError("compactedLedgers[ctx]")
        return led[ctx - 1]

    def inv(self, name, s):
        if self.user is not None and name in self.user.defs:
            import tla_eval
            try:
                return self.user.holds(name, s)
            except tla_eval.EvalError as e:
                raise EvalError(str(e))
        msgs, led, cur, ph, p1r, hz, ctx, crash, cons = s
        N, C = self.N, self.C
        if name == "TypeSafe":  # :236-248
            def ok(m):
                return 1 <= m[0] <= N and m[1] in self.keyset and m[2] in self.valueset
            if not all(ok(m) for m in msgs):
                return False
            if not all(l is None or all(ok(m) for m in l) for l in led):
                return False
            if p1r is not None:
                if not all(1 <= v <= len(msgs) for _, v in p1r[1]) or not 1 <= p1r[0] <= len(msgs):
                    return False
            return (0 <= ph < 6 and 0 <= hz <= N and 0 <= ctx <= C and 0 <= crash <= self.K
                    and (cur is None or (1 <= cur[0] <= N and 1 <= cur[1] <= C)))
        if name == "CompactedLedgerLeak":  # :253
            return sum(l is not None for l in led) <= 2
        if name == "CompactionHorizonCorrectness":  # :259-274, literally
            # Len(messagesBeforeHorizon) (:269) enumerates the function, so every
            # messages[i], i <= hz, is evaluated before the first i is tested
            if hz > len(msgs):
                raise EvalError("messages[i]")
            for i in range(1, hz + 1):
                m = msgs[i - 1]
                if m[1] == 0 and not self.retain:
                    continue  # messagesBeforeHorizon[i] = Nil: FALSE => ... holds (:271)
                L = self.ledger_at_ctx(s)
                # ELSE branch (:272-274), a retained null-key message included
                if not any(e[1] == m[1] and e[0] >= m[0] for e in L):
                    return False
            return True
        if name == "DuplicateNullKeyMessage":  # :280-294
            if not (self.retain and ctx != 0):
                return True
            L = self.ledger_at_ctx(s)
            after = msgs[hz:]
            return all(e[1] != 0 or all(e != m for m in after) for e in L)
        raise ValueError(name)

    def check(self):
        """TLC -workers 1 BFS. Returns a dict like tlc_oracle's JSON."""
        seen, parent = {}, []
        states, levels, generated = [], [], 0

        def add(t, par, act):
            if t in seen:
                return None
            seen[t] = len(states)
            states.append(t)
            parent.append((par, act))
            return len(states) - 1

        def bad(t):
            for name in self.invariants:
                try:
                    if not self.inv(name, t):
                        return ("invariant", name)
                except EvalError:
                    return ("invariant_error", name)
            return None

        def trace(k, extra=None):
            out = []
            while k is not None and k >= 0:
                out.append((parent[k][1], states[k]))
                k = parent[k][0]
            out.reverse()
            if extra:
                out.append(extra)
            return out

        def end_of_level(first, last):
            """The counts of a level-synchronous checker that finishes the level
            [first, last) it was expanding: every state expanded, every successor
            of every action that does not fail counted and inserted."""
            gen = gen_at_level
            for q in range(first, last):
                succ = []
                try:
                    for x in self.successors(states[q]):
                        succ.append(x)
                except EvalError:  # a failing compactor disjunct: the later ones still run
                    succ += list(self.tail_actions(states[q]))
                gen += len(succ)
                for a, t in succ:
                    add(t, q, ACTIONS[a])
            return gen, len(states)

        gen_at_level = 0
        for t in self.inits():
            generated += 1
            k = add(t, -1, "Init")
            if k is not None:
                b = bad(t)
                if b:
                    r = dict(result=b[0], invariant=b[1], generated=generated, distinct=len(states),
                             left_on_queue=len(states), trace=trace(k))
                    for t2 in self.inits():  # end of level 0: every initial state
                        add(t2, -1, "Init")
                    r["eol_generated"], r["eol_distinct"] = sum(1 for _ in self.inits()), len(states)
                    return r
        levels.append(len(states))
        outdeg = {}  # new states discovered per expanded state (TLC's outdegree statistics)
        head = 0
        while head < len(states):
            end = len(states)
            gen_at_level = generated
            for p in range(head, end):
                s = states[p]
                n = 0

                def stop(**kw):  # TLC's counters when the run stops while expanding p
                    r = dict(generated=generated, distinct=len(states), left_on_queue=len(states) - (p + 1), **kw)
                    r["eol_generated"], r["eol_distinct"] = end_of_level(head, end)
                    return r

                def process(group):
                    """one action's successors: counted as a whole (TLC's StateVec),
                    then inserted and checked one by one"""
                    nonlocal generated, n
                    generated += len(group)
                    n += len(group)
                    for a, t in group:
                        k = add(t, p, ACTIONS[a])
                        if k is not None:
                            b = bad(t)
                            if b:
                                return stop(result=b[0], invariant=b[1], trace=trace(k))
                    return None

                n_before = len(states)
                pending = []
                try:
                    for a, t in self.successors(s):
                        if pending and pending[0][0] != a:
                            r = process(pending)
                            if r:
                                return r
                            pending = []
                        pending.append((a, t))
                except EvalError:
                    return stop(result="action_error", trace=trace(p))
                r = process(pending)
                if r:
                    return r
                if n == 0 and self.deadlock:
                    return stop(result="deadlock", trace=trace(p))
                k_new = len(states) - n_before
                outdeg[k_new] = outdeg.get(k_new, 0) + 1
            head = end
            if len(states) > end:
                levels.append(len(states) - end)
        hist = [outdeg.get(i, 0) for i in range(max(outdeg) + 1)] if outdeg else []
        return dict(result="ok", generated=generated, distinct=len(states), depth=len(levels), levels=levels,
                    outdegree=hist)

    # ---- PROPERTY Termination, compaction.tla:303-307 ----
    def termination_p(self, s):
        """Termination's state predicate P (<>P), the guard of Terminating."""
        msgs, led, cur, ph, p1r, hz, ctx, crash, cons = s
        return (len(msgs) == self.N and ph == W and self.max_ledger(led) == self.C
                and (not self.consumer or cons == self.ctl))

    def liveness(self, fair):
        """<>P under Spec (fair=False: every behavior may stutter forever) or
        Spec /\\ WF_vars(Next) (fair=True).  Counterexamples live in G', the
        states reachable from Init through not-P states.  Under WF a behavior
        stutters forever only where every successor equals the state ("stuck"),
        else it takes non-stuttering steps forever: <>P fails iff G' has a stuck
        state or a cycle.  The cycle test here is a depth-first search for a
        back edge (white/grey/black colouring) -- a third algorithm beside the C
        oracle's Tarjan SCC and the GPU's Kahn peeling."""
        index, states, depth, adj = {}, [], [], []
        q = deque()
        for t in self.inits():
            if not self.termination_p(t) and t not in index:
                index[t] = len(states)
                states.append(t)
                depth.append(1)
                q.append(index[t])
        edges, stuck, stuck_depth = 0, 0, None
        while q:
            k = q.popleft()
            s = states[k]
            moves, out = 0, []
            for _, t in self.successors(s):
                if t == s:
                    continue  # a stutter
                moves += 1
                if self.termination_p(t):
                    continue
                if t not in index:
                    index[t] = len(states)
                    states.append(t)
                    depth.append(depth[k] + 1)
                    q.append(index[t])
                out.append(index[t])
            edges += len(out)
            adj.append(out)
            if moves == 0 or not fair:
                stuck += 1
                if stuck_depth is None:
                    stuck_depth = depth[k]
        colour = [0] * len(states)  # 0 white, 1 grey (on the DFS path), 2 black
        cyclic = False
        for r in range(len(states)):
            if colour[r] or cyclic:
                continue
            stack = [(r, 0)]
            colour[r] = 1
            while stack and not cyclic:
                v, i = stack[-1]
                if i < len(adj[v]):
                    stack[-1] = (v, i + 1)
                    w = adj[v][i]
                    if colour[w] == 1:
                        cyclic = True
                    elif colour[w] == 0:
                        colour[w] = 1
                        stack.append((w, 0))
                else:
                    colour[v] = 2
                    stack.pop()
        return dict(holds=stuck == 0 and not cyclic, states_notp=len(states),
                    init_notp=sum(1 for d in depth if d == 1), edges_notp=edges, stuck=stuck,
                    stuck_min_depth=stuck_depth or 0, cyclic=cyclic)
