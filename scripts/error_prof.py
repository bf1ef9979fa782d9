"""One erroring P8 check (the ledger-leak reproducer on the Producer tree),
reported as TLC reports it, REPS times: for rocprofv3 --kernel-trace --stats
(the subtree run's kernels against its wall time).

    python scripts/error_prof.py [REPS]
"""
import os
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "pulsar-tlaplus_amd", "python"))
sys.path.insert(0, ROOT)
import tlcgpu as T  # noqa: E402
from bench import model_for  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
m = model_for("p8")
bad = T.Model(**{**m.__dict__, "invariants": ("TypeSafe", "CompactedLedgerLeak")})
ck = T.Checker(bad)
for i in range(reps + 1):
    t0 = time.perf_counter()
    r = ck.run()
    stop = ck.tlc_stop_stats()
    print(i, r.engine, r.status, r.depth, stop, round((time.perf_counter() - t0) * 1e3, 3), "ms", flush=True)
ck.close()
