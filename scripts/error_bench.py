"""Wall time of a check that stops on an error, reported as TLC reports it
(VERDICT r3 item 6): the default engine's run plus the trace and TLC's stop
counters (tlcg_tlc_stop_stats), against the same engine's clean check of the
same constants.  One JSON line per case.

    python scripts/error_bench.py [REPS]

Cases: P8 (the component tree, Producer modelled) with the ledger-leak
reproducer CompactedLedgerLeak (compaction.cfg:27-28); G9 (the component
engine) with it; P8 and G9 with an injected user invariant violated at depth
(LedgerCount <= 2, BASELINE config 5)."""
import json
import os
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "pulsar-tlaplus_amd", "python"))
sys.path.insert(0, ROOT)
import tlcgpu as T  # noqa: E402
from bench import model_for  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
LEDGER_COUNT = "Cardinality({i \\in 1..CompactionTimesLimit : compactedLedgers[i] # Nil}) <= 2"


def with_invariants(m, invariants, user=None):
    return T.Model(**{**m.__dict__, "invariants": invariants, "user_defs": user})


cases = []
for cfg in ("p8", "g9"):
    clean = model_for(cfg)
    cases.append((f"{cfg}_leak", clean, with_invariants(clean, ("TypeSafe", "CompactedLedgerLeak"))))
    cases.append((f"{cfg}_user_ledgercount", clean,
                  with_invariants(clean, ("TypeSafe", "LedgerCount"), {"LedgerCount": LEDGER_COUNT})))

for name, clean, bad in cases:
    ck = T.Checker(clean)
    ck.run(with_trace=False)  # (warm: hipRTC module, buffers)
    t_clean = []
    for _ in range(reps):
        t0 = time.perf_counter()
        r0 = ck.run(with_trace=False)
        t_clean.append(time.perf_counter() - t0)
    ck.close()
    ck = T.Checker(bad)
    r = ck.run()
    ck.tlc_stop_stats()
    t_err = []
    for _ in range(reps):
        t0 = time.perf_counter()
        r = ck.run()  # (the trace included)
        stop = ck.tlc_stop_stats()
        t_err.append(time.perf_counter() - t0)
    ck.close()
    print(json.dumps(dict(case=name, clean_engine=r0.engine, clean_s=round(min(t_clean), 5),
                          error_engine=r.engine, status=r.status, invariant=r.invariant, depth=r.depth,
                          tlc_exact=r.tlc_exact, trace_len=len(r.trace), stop=list(stop),
                          eol=[r.generated, r.distinct], error_s=round(min(t_err), 5),
                          ratio=round(min(t_err) / min(t_clean), 2))), flush=True)
