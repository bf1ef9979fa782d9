"""GPU: the distributed level loop (dist.run) with real libtlcgpu engines in
separate processes, one rank per process, all on cuda:0.  RCCL refuses two
ranks on one device ("Duplicate GPU detected", profiles/r01_rccl_probe.log),
so the records travel over gloo through host memory here; the driver's
8-GPU run takes the same code path with the nccl backend over xGMI."""
import json
import os
import socket

import pytest
import torch.multiprocessing as mp

from conftest import GOLDEN, model_of

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, case, partition, outdir):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    sys.path.insert(0, os.path.join(os.path.dirname(here), "pulsar-tlaplus_amd", "python"))
    import torch.distributed as dist
    import dist as tdist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        eng = tdist.GpuEngine(model_of(GOLDEN[case]["constants"]), rank, world, 0, partition=partition)
        timing = {}
        r = tdist.run(eng, timing=timing)
        eng.close()
        with open(os.path.join(outdir, f"r{rank}.json"), "w") as f:
            json.dump(dict(status=r.status, generated=r.generated, distinct=r.distinct, depth=r.depth,
                           levels=r.levels, closed=r.closed, invariant=r.invariant), f)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("case,partition,world", [("S", 2, 2), ("P_published", 0, 2), ("P_published", 0, 3),
                                                  ("X_keys3_vals57", 2, 3), ("S", 0, 2),
                                                  ("V_leak", 0, 2), ("V_leak", 2, 3), ("V_dup", 0, 3),
                                                  ("V_dup", 2, 2), ("V_leak_producer", 0, 2)])
def test_gpu_ranks_match_single(tmp_path, case, partition, world):
    mp.spawn(_worker, args=(world, _free_port(), case, partition, str(tmp_path)), nprocs=world, join=True)
    want = GOLDEN[case]["result"]
    c = GOLDEN[case]["constants"]
    for rank in range(world):
        r = json.load(open(tmp_path / f"r{rank}.json"))
        assert r["closed"] == (partition != 2 and not c["producer"])
        assert r["status"] == want["result"]
        if want["result"] == "ok":
            assert (r["generated"], r["distinct"], r["depth"], r["levels"]) == (
                want["generated"], want["distinct"], want["depth"], want["levels"])
        else:  # the first error (lowest level, then rank); counts at the end of its level
            assert c["invariants"][r["invariant"]] == want["invariant"]
            assert (r["generated"], r["distinct"], r["depth"]) == (
                want["eol_generated"], want["eol_distinct"], want["depth"])
            assert r["levels"][:-1] == want["levels"][:-1] and sum(r["levels"]) == want["eol_distinct"]
