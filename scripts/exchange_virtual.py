"""Timing of the open-partition level loop with W virtual ranks on one GPU
(W contexts, device-copy exchange): expand / absorb device time per rank and
wall time per check.  TLCG_LIB selects the library build (A/B)."""
import json, os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'pulsar-tlaplus_amd', 'python'))
import torch
import dist as tdist
import tlcgpu
W = int(sys.argv[1]) if len(sys.argv) > 1 else 8
k = int(sys.argv[2]) if len(sys.argv) > 2 else 15
m = tlcgpu.Model(key_space=range(1, k + 1), value_space=range(1, k + 1))
n = 62 * (k + 1) ** 6
per = n // W + 1
engines = [tdist.GpuEngine(m, r, W, 0, partition=2, log2_fpset_slots=max(16, (2 * per - 1).bit_length()),
                           state_capacity=int(per * 1.1) + (1 << 20)) for r in range(W)]
for rep in range(2):
    t0 = time.perf_counter()
    stats = [e.init() for e in engines]
    xs = 0.0
    while sum(e.level_sizes()[-1] for e in engines):
        for e in engines:
            e.expand()
        t1 = time.perf_counter()
        for dst in range(W):
            parts = [engines[src].outbox(dst) for src in range(W) if src != dst]
            recs = torch.cat(parts, 0)
            if recs.shape[0]:
                engines[dst].absorb(recs)
        xs += time.perf_counter() - t1
        stats = [e.end_level() for e in engines]
    wall = time.perf_counter() - t0
    d = sum(s.distinct for s in stats)
    print(json.dumps(dict(world=W, distinct=d, wall_s=round(wall, 3), exchange_s=round(xs, 3),
                          expand_ms_per_rank=[round(s.expand_ms, 2) for s in stats],
                          kernel_ms_per_rank=[round(s.kernel_ms, 2) for s in stats])), flush=True)
for e in engines:
    e.close()
