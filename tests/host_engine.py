"""TEST INFRASTRUCTURE: a CPU stand-in for one rank of libtlcgpu's partitioned
API, built on the product's host-compiled successor function
(tlcg_host_successors).  It lets tests drive the distributed level loop
(pulsar-tlaplus_amd/python/dist.py) over gloo on CPU.  Never used by the
product path."""
from types import SimpleNamespace

import torch

import tlcgpu


def _mix64(x):
    m = (1 << 64) - 1
    x ^= x >> 33
    x = (x * 0xff51afd7ed558ccd) & m
    x ^= x >> 33
    x = (x * 0xc4ceb9fe1a85ec53) & m
    x ^= x >> 33
    return x


class HostEngine:
    def __init__(self, model, rank, world, closed):
        self.m, self.rank, self.world, self.closed = model, rank, world, closed
        self.seen, self.levels, self.frontier = set(), [], []
        self.gen = 0
        self.status = 0
        self.out = [[] for _ in range(world)]
        self.pending = []

    def owner(self, s):
        return ((_mix64(s) >> 32) * self.world) >> 32

    def _stats(self):
        return SimpleNamespace(generated=self.gen, distinct=len(self.seen), status=self.status, kernel_ms=0.0,
                               expand_ms=0.0)

    def _add(self, t):
        if t in self.seen:
            return
        self.seen.add(t)
        self.pending.append(t)
        if tlcgpu.host_check_invariants(self.m, t) >= 0:
            self.status = 2

    def init(self):
        n = tlcgpu.init_count(self.m)
        for i in range(n):
            s = tlcgpu.host_init_state(self.m, i)
            mine = (i % self.world == self.rank) if self.closed else self.owner(s) == self.rank
            if mine:
                self.gen += 1
                self._add(s)
        self._commit()
        return self._stats()

    def _commit(self):
        self.levels.append(len(self.pending))
        self.frontier, self.pending = self.pending, []

    def expand(self):
        self.out = [[] for _ in range(self.world)]
        for s in self.frontier:
            succ = tlcgpu.host_successors(self.m, s)
            if not succ and self.m.check_deadlock:
                self.status = 3
            for _, t in succ:
                self.gen += 1
                d = self.rank if self.closed else self.owner(t)
                if d == self.rank:
                    self._add(t)
                else:
                    self.out[d].append((t, self.rank << 56))
        return [len(o) if d != self.rank else 0 for d, o in enumerate(self.out)]

    def outbox(self, d):
        return torch.tensor(self.out[d], dtype=torch.int64).reshape(-1, 2)

    def absorb(self, recs):
        for t, _ in recs.tolist():
            self._add(t)

    def end_level(self):
        self._commit()
        return self._stats()

    def run_closed(self):
        self.init()
        while self.frontier and self.status == 0:
            self.expand()
            self.end_level()
        if self.levels and self.levels[-1] == 0:
            self.levels.pop()
        return self._stats()

    def level_sizes(self):
        return list(self.levels)

    def new_tensor(self, shape, dtype):
        return torch.empty(shape, dtype=dtype)
