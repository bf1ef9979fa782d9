"""First on-GPU check: parity with the oracle's published/derived counts + a G9 timing."""
import sys, time, json, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'pulsar-tlaplus_amd', 'python'))
import tlcgpu as T
def show(name, r):
    print(name, json.dumps(dict(status=r.status, gen=r.generated, dist=r.distinct, depth=r.depth, inv=r.invariant,
          trace=[a for a,_ in r.trace], kms=round(r.kernel_ms,3), redone=r.levels_redone)), flush=True)
show("S", T.run(T.Model()))
show("S-tlc", T.run(T.Model(), tlc_order=True))
show("P", T.run(T.Model(model_producer=True, retain_null_key=False)))
show("P-tlc", T.run(T.Model(model_producer=True, retain_null_key=False), tlc_order=True))
show("leak", T.run(T.Model(invariants=("TypeSafe","CompactedLedgerLeak","CompactionHorizonCorrectness"))))
show("leak-tlc", T.run(T.Model(invariants=("TypeSafe","CompactedLedgerLeak","CompactionHorizonCorrectness")), tlc_order=True))
show("dup-tlc", T.run(T.Model(invariants=("TypeSafe","CompactionHorizonCorrectness","DuplicateNullKeyMessage")), tlc_order=True))
m8 = T.Model(key_space=range(1,11), value_space=range(1,11))
t=time.time(); show("M8", T.run(m8)); print("wall", time.time()-t)
g9 = T.Model(key_space=range(1,16), value_space=range(1,16))
ck = T.Checker(g9, log2_fpset_slots=31, state_capacity=1_200_000_000)
for i in range(3):
    t=time.time(); ck.run_raw(); dt=time.time()-t
    r = ck.result(False); show("G9", r); print("wall", dt, "distinct/s", r.distinct/dt, flush=True)
