"""CPU: the distributed level loop (dist.py) with world_size 2 and 3 over gloo,
both partition regimes, against the golden single-process counts."""
import json
import os
import socket

import pytest
import torch.multiprocessing as mp

from conftest import GOLDEN, model_of


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class FakeEngine:
    """A closed-partition rank with canned results (the combine logic alone)."""
    closed = True

    def __init__(self, status, levels, gen, invariant=-1):
        from types import SimpleNamespace
        self.st = SimpleNamespace(status=status, generated=sum(gen), distinct=sum(levels), kernel_ms=0.0,
                                  expand_ms=0.0, invariant=invariant)
        self.levels, self.gen = levels, gen

    def run_closed(self):
        return self.st

    def level_sizes(self):
        return list(self.levels)

    def level_generated(self):
        return list(self.gen)


# rank 0 deadlocks while expanding level 9 (depth 10); rank 1 violates invariant 1
# at level 1 (depth 2), having expanded only level 0; rank 2 runs out at depth 5
FAKE = [dict(status=3, levels=[4] * 10, gen=[4] + [5] * 10),
        dict(status=2, levels=[3, 6], gen=[3, 7], invariant=1),
        dict(status=1, levels=[2, 2, 2, 2, 2], gen=[2, 3, 3, 3, 3, 3])]


def _fake_worker(rank, world, port, outdir):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(os.path.dirname(here), "pulsar-tlaplus_amd", "python"))
    import torch.distributed as dist
    import dist as tdist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        r = tdist.run(FakeEngine(**FAKE[rank]))
        with open(os.path.join(outdir, f"r{rank}.json"), "w") as f:
            json.dump(dict(status=r.status, generated=r.generated, distinct=r.distinct, depth=r.depth,
                           levels=r.levels, invariant=r.invariant, first=r.first_error_rank), f)
    finally:
        dist.destroy_process_group()


def test_first_error_is_lowest_level_then_rank(tmp_path):
    """the combined verdict is the error in the lowest level (then
    the lowest rank), not the largest status code, and every rank's counts are
    cut at the end of that level (levels 0..1 here, generated up to them)."""
    mp.spawn(_fake_worker, args=(3, _free_port(), str(tmp_path)), nprocs=3, join=True)
    for rank in range(3):
        r = json.load(open(tmp_path / f"r{rank}.json"))
        assert (r["status"], r["depth"], r["first"], r["invariant"]) == ("invariant", 2, 1, 1)
        assert r["levels"] == [4 + 3 + 2, 4 + 6 + 2]
        assert r["distinct"] == 21
        assert r["generated"] == (4 + 5) + (3 + 7) + (2 + 3)


def _worker(rank, world, port, case, closed, outdir):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    sys.path.insert(0, os.path.join(os.path.dirname(here), "pulsar-tlaplus_amd", "python"))
    import torch.distributed as dist
    import dist as tdist
    from host_engine import HostEngine
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        eng = HostEngine(model_of(GOLDEN[case]["constants"]), rank, world, closed)
        r = tdist.run(eng)
        with open(os.path.join(outdir, f"r{rank}.json"), "w") as f:
            json.dump(dict(status=r.status, generated=r.generated, distinct=r.distinct, depth=r.depth,
                           levels=r.levels), f)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("case,closed,world", [("S", True, 2), ("S", False, 2), ("X_producer_sparse", False, 2),
                                               ("X_producer_sparse", False, 3), ("X_keys3_vals57", True, 3),
                                               ("V_leak", True, 2), ("V_leak", False, 3), ("V_dup", True, 3),
                                               ("V_dup", False, 2)])
def test_dist_matches_single(tmp_path, case, closed, world):
    mp.spawn(_worker, args=(world, _free_port(), case, closed, str(tmp_path)), nprocs=world, join=True)
    want = GOLDEN[case]["result"]
    for rank in range(world):
        r = json.load(open(tmp_path / f"r{rank}.json"))
        assert r["status"] == want["result"]
        if want["result"] == "ok":
            assert (r["generated"], r["distinct"], r["depth"], r["levels"]) == (
                want["generated"], want["distinct"], want["depth"], want["levels"])
        else:  # end of the error's level, as one context reports it
            assert (r["generated"], r["distinct"], r["depth"]) == (
                want["eol_generated"], want["eol_distinct"], want["depth"])
            assert r["levels"][:-1] == want["levels"][:-1] and sum(r["levels"]) == want["eol_distinct"]
