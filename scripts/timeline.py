"""Device timeline of a rocprofv3 --kernel-trace CSV: for each check (a
check starts at the first kernel whose name holds MARK, default k_init), the
span from its first kernel's start to its last kernel's end, the union of
busy intervals (any kernel running), each kernel class's own union, and the
idle time (span - busy).  Used on node_bench runs (several ranks' streams on
one GPU) to tell device work from the gaps the level loop's host syncs leave.

    python scripts/timeline.py run_kernel_trace.csv [MARK]
"""
import csv
import json
import re
import sys


def union(iv):
    iv = sorted(iv)
    tot, cur_s, cur_e = 0, None, None
    for s, e in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def short(name):
    m = re.search(r"(k_[A-Za-z0-9_]+|tlcg_[A-Za-z0-9_]+|__amd_rocclr_[A-Za-z]+|nccl[A-Za-z0-9_]+)", name)
    return m.group(1) if m else name[:40]


def main():
    path = sys.argv[1]
    mark = sys.argv[2] if len(sys.argv) > 2 else "k_init"
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    # a check: from one cluster of MARK kernels to the next (the ranks' inits come together)
    starts = []
    for s, e, k in rows:
        if mark in k and (not starts or s - starts[-1] > 5e6):
            starts.append(s)
    bounds = starts + [float("inf")]
    for i in range(len(starts)):
        seg = [r for r in rows if bounds[i] <= r[0] < bounds[i + 1]]
        if not seg:
            continue
        t0 = seg[0][0]
        t1 = max(e for _, e, _ in seg)
        busy = union([(s, e) for s, e, _ in seg])
        per = {}
        for s, e, k in seg:
            per.setdefault(k, []).append((s, e))
        out = dict(check=i, span_ms=round((t1 - t0) / 1e6, 3), busy_ms=round(busy / 1e6, 3),
                   idle_ms=round((t1 - t0 - busy) / 1e6, 3), kernels=len(seg),
                   classes={k: dict(n=len(v), union_ms=round(union(v) / 1e6, 3),
                                    sum_ms=round(sum(e - s for s, e in v) / 1e6, 3))
                            for k, v in sorted(per.items(), key=lambda kv: -union(kv[1]))})
        print(json.dumps(out))


if __name__ == "__main__":
    main()
