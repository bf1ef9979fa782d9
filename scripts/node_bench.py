"""Wall time of tlcg_run_node (tlc-hip -gpus N's path) on G9 with the FPSet
partitioned on the whole state (BASELINE config 4) at W ranks on the GPUs of
this host; on one GPU the ranks share it (local transport)."""
import json, os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "pulsar-tlaplus_amd", "python"))
import tlcgpu
W = int(sys.argv[1]) if len(sys.argv) > 1 else 8
k = int(sys.argv[2]) if len(sys.argv) > 2 else 15
m = tlcgpu.Model(key_space=range(1, k + 1), value_space=range(1, k + 1))
per = 62 * (k + 1) ** 6 // W + 1
for rep in range(3):
    t0 = time.perf_counter()
    r = tlcgpu.run_node(m, W, partition=2, engine="global", log2_fpset_slots=(2 * per - 1).bit_length(),
                        state_capacity=int(per * 1.1) + (1 << 20))
    wall = time.perf_counter() - t0
    print(json.dumps(dict(world=W, keys=k, distinct=r.distinct, generated=r.generated, depth=r.depth,
                          transport=r.transport, wall_s=round(wall, 3), kernel_ms_max_rank=round(r.kernel_ms, 2),
                          expand_ms_max_rank=round(r.expand_ms, 2))), flush=True)
