"""Diagnostics (CPU, no GPU): write the hipRTC source of the kernels
specialized for a cfg (TLCG_JIT_DUMP) and compile it offline with hipcc to
gfx950 assembly, so the ISA of the specialized kernels can be read.

    python scripts/jit_isa.py [keys|cfg] [out_prefix]   -> out_prefix.hip, out_prefix.s

keys: KeySpace = ValueSpace = 1..keys (G9's constants otherwise); cfg: one
of bench.py's CONFIGS (s, m8, g9, g9deep, p8).
"""
import ctypes as C
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pulsar-tlaplus_amd", "python"))
import tlcgpu  # noqa: E402

arg = sys.argv[1] if len(sys.argv) > 1 else "15"
out = sys.argv[2] if len(sys.argv) > 2 else "/tmp/g9jit"
os.environ["TLCG_JIT_DUMP"] = out + ".hip"
os.environ["TLCG_JIT_CACHE"] = "/tmp/tlcg-jit-isa-nocache"
if arg.isdigit():
    m = tlcgpu.Model(key_space=range(1, int(arg) + 1), value_space=range(1, int(arg) + 1))
else:
    sys.path.insert(0, ROOT)
    from bench import model_for  # noqa: E402
    m = model_for(arg)
cm = m.to_c()
err = C.create_string_buffer(8192)
n = tlcgpu.load_library().tlcg_jit_selftest(C.byref(cm), b"gfx950", err, 8192)
if n < 0:
    raise SystemExit(err.value.decode())
opts = os.environ.get("TLCG_JIT_OPTS", "-mllvm -amdgpu-sched-strategy=max-ilp").split()
# the dumped source holds the headers inline; its own #include lines resolve to empty stubs
import re  # noqa: E402
stub = out + "_inc"
os.makedirs(stub, exist_ok=True)
for h in set(re.findall(r'#include "([^"]+)"', open(out + ".hip").read())):
    open(os.path.join(stub, h), "w").close()
subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++20", "-x", "hip", "--cuda-device-only",
                "-S", "-I" + stub, "-o", out + ".s", out + ".hip"] + opts, check=True)
print(out + ".s")
# the wave kernels' module (jit.cpp JIT_WAVE: the default scheduler unless TLCG_JIT_OPTS_WAVE)
if os.path.exists(out + ".hip.wave"):
    wopts = os.environ.get("TLCG_JIT_OPTS_WAVE", "").split()
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++20", "-x", "hip",
                    "--cuda-device-only", "-S", "-I" + stub, "-x", "hip", "-o", out + ".wave.s",
                    out + ".hip.wave"] + wopts, check=True)
    print(out + ".wave.s")
