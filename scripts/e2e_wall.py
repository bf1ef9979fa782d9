"""End-to-end process wall of one complete model check through the C-ABI
("BFS wall ... plus end-to-end process wall").

For each cfg the parent starts a fresh child process and times it from spawn to
exit; the child reports its own phases: interpreter + library load, tlcg_create
(device buffers), a first tlcg_init (hipRTC specialization on a cold cache +
Init), tlcg_run (Init again + the BFS), and the result read-back.  `cold` runs
use an empty TLCG_JIT_CACHE, `warm` runs the cache the cold run filled.  The `tlc-hip` CLI cannot run on the GPU box
(the spec text is not shipped there), so this is the same path minus cfg parsing.

    python scripts/e2e_wall.py [cfg ...]        (default: s p8 m8 g9)
"""
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(cfg):
    t0 = time.perf_counter()
    sys.path.insert(0, ROOT)
    import bench
    import tlcgpu
    tlcgpu.load_library()
    model = bench.model_for(cfg)
    t1 = time.perf_counter()
    ck = tlcgpu.Checker(model, device=0)
    t2 = time.perf_counter()
    st = ck.init()
    t3 = time.perf_counter()
    ck.run_raw()
    t4 = time.perf_counter()
    r = ck.result(with_trace=False)
    t5 = time.perf_counter()
    ck.close()
    want = bench.CONFIGS[cfg]
    ok = (r.generated, r.distinct, r.depth) == (want["generated"], want["distinct"], want["depth"])
    print(json.dumps(dict(cfg=cfg, ok=ok, distinct=r.distinct, generated=r.generated, depth=r.depth,
                          engine=tlcgpu.ENGINE_NAMES.get(int(st.engine), "?"), jit=int(st.jit_used),
                          load_s=round(t1 - t0, 3), create_s=round(t2 - t1, 3), first_init_s=round(t3 - t2, 3),
                          check_s=round(t4 - t3, 4), result_s=round(t5 - t4, 4), close_s=round(time.perf_counter() - t5, 3))))


def main(cfgs):
    cache = tempfile.mkdtemp(prefix="tlcg-jit-e2e-")
    env = dict(os.environ, TLCG_JIT_CACHE=cache)
    bad = 0
    for cfg in cfgs:
        for mode in ("cold", "warm"):
            if mode == "cold":
                for f in os.listdir(cache):
                    os.remove(os.path.join(cache, f))
            t0 = time.perf_counter()
            p = subprocess.run([sys.executable, "-u", os.path.abspath(__file__), "--child", cfg], env=env,
                               capture_output=True, text=True, timeout=300)
            wall = time.perf_counter() - t0
            if p.returncode != 0:
                print(json.dumps(dict(cfg=cfg, mode=mode, rc=p.returncode, err=p.stderr[-800:])), flush=True)
                return 1
            rec = json.loads(p.stdout.strip().splitlines()[-1])
            rec.update(mode=mode, process_wall_s=round(wall, 3),
                       distinct_per_s_e2e=round(rec["distinct"] / wall, 1))
            bad += not rec["ok"]
            print(json.dumps(rec), flush=True)
    return 1 if bad else 0


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        child(sys.argv[2])
    else:
        sys.exit(main(sys.argv[1:] or ["s", "p8", "m8", "g9"]))
