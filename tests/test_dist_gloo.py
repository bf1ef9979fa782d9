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
                                               ("X_producer_sparse", False, 3), ("X_keys3_vals57", True, 3)])
def test_dist_matches_single(tmp_path, case, closed, world):
    mp.spawn(_worker, args=(world, _free_port(), case, closed, str(tmp_path)), nprocs=world, join=True)
    want = GOLDEN[case]["result"]
    for rank in range(world):
        r = json.load(open(tmp_path / f"r{rank}.json"))
        assert r["status"] == want["result"]
        assert (r["generated"], r["distinct"], r["depth"], r["levels"]) == (
            want["generated"], want["distinct"], want["depth"], want["levels"])
