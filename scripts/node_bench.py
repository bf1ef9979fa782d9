"""Wall time of the node-level check (tlc-hip -gpus N's path, tlcg_node_*) on
G9 with the FPSet partitioned on the whole state (BASELINE config 4) at W
ranks on the GPUs of this host; on one GPU the ranks share it (local
transport).  The ranks' contexts are built once (create_s) and every check
reuses them (wall_s: one complete check, the level loop and the combine).

    python scripts/node_bench.py [W] [KEYS] [CHECKS]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "pulsar-tlaplus_amd", "python"))
import tlcgpu  # noqa: E402

W = int(sys.argv[1]) if len(sys.argv) > 1 else 8
k = int(sys.argv[2]) if len(sys.argv) > 2 else 15
checks = int(sys.argv[3]) if len(sys.argv) > 3 else 5
m = tlcgpu.Model(key_space=range(1, k + 1), value_space=range(1, k + 1))
per = 62 * (k + 1) ** 6 // W + 1
t0 = time.perf_counter()
node = tlcgpu.Node(m, W, partition=2, engine="global", log2_fpset_slots=(2 * per - 1).bit_length(),
                   state_capacity=int(per * 1.1) + (1 << 20))
create_s = time.perf_counter() - t0
for rep in range(checks):
    t0 = time.perf_counter()
    r = node.run()
    wall = time.perf_counter() - t0
    print(json.dumps(dict(world=W, keys=k, check=rep, distinct=r.distinct, generated=r.generated, depth=r.depth,
                          levels_redone=r.levels_redone, transport=r.transport, create_s=round(create_s, 3),
                          wall_s=round(wall, 4), kernel_ms_max_rank=round(r.kernel_ms, 2),
                          expand_ms_max_rank=round(r.expand_ms, 2))), flush=True)
t0 = time.perf_counter()
node.close()
print(json.dumps(dict(world=W, destroy_s=round(time.perf_counter() - t0, 3))), flush=True)
