"""CPU: libtlcgpu.so loads, exports every entry point include/tlcgpu.h
declares, validates models, and refuses to run without a GPU (no fallback)."""
import ctypes
import ctypes as C
import os
import re

import pytest

import tlcgpu
from conftest import LIB, ROOT


def declared_functions():
    with open(os.path.join(ROOT, "include", "tlcgpu.h")) as f:
        text = f.read()
    return sorted(set(re.findall(r"\b(tlcg_[a-z_0-9]+)\s*\(", text)))


def test_header_declares_the_boundary():
    names = declared_functions()
    for required in ("tlcg_create", "tlcg_init", "tlcg_step_level", "tlcg_run", "tlcg_trace", "tlcg_decode",
                     "tlcg_destroy", "tlcg_last_error", "tlcg_expand", "tlcg_absorb"):
        assert required in names


def test_every_declared_symbol_is_exported():
    lib = ctypes.CDLL(LIB)
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing


def test_python_binding_covers_the_header():
    lib = tlcgpu.load_library()
    for n in declared_functions():
        assert getattr(lib, n).argtypes is not None or getattr(lib, n).restype is not None, n


def test_abi_version():
    assert tlcgpu.load_library().tlcg_abi_version() == 4


def test_struct_layout_matches_c(tmp_path):
    # every field offset of the ctypes mirrors == what the C compiler lays out
    import subprocess
    structs = [tlcgpu.tlcg_model, tlcgpu.tlcg_opts, tlcgpu.tlcg_stats, tlcgpu.tlcg_liveness]
    src = ['#include <stdio.h>', '#include <stddef.h>', '#include "tlcgpu.h"', "int main(void){"]
    for st in structs:
        src.append(f'printf("%zu\\n", sizeof({st.__name__}));')
        for name, _ in st._fields_:
            src.append(f'printf("%zu\\n", offsetof({st.__name__}, {name}));')
    src.append("return 0;}")
    (tmp_path / "l.c").write_text("\n".join(src))
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), "-o", str(tmp_path / "l"), str(tmp_path / "l.c")],
                   check=True)
    got = [int(x) for x in subprocess.run([str(tmp_path / "l")], capture_output=True, text=True).stdout.split()]
    want = []
    for st in structs:
        want.append(ctypes.sizeof(st))
        want += [getattr(st, name).offset for name, _ in st._fields_]
    assert got == want


@pytest.mark.parametrize("kw,msg", [
    (dict(key_space=[0, 1]), "0 \\notin KeySpace"),
    (dict(value_space=[0]), "0 \\notin ValueSpace"),
    (dict(key_space=[-1]), "KeySpace \\in SUBSET Nat"),
    (dict(msg_sent_limit=-1), "MessageSentLimit \\in Nat"),
    (dict(max_crash_times=-2), "MaxCrashTimes \\in Nat"),
    (dict(compaction_times_limit=30, key_space=range(1, 11), value_space=range(1, 11)), "126 bits"),
])
def test_check_model_rejects(kw, msg):
    err = tlcgpu.check_model(tlcgpu.Model(**kw))
    assert err is not None and msg in err


def test_check_model_accepts_scaled():
    assert tlcgpu.check_model(tlcgpu.Model(key_space=range(1, 16), value_space=range(1, 16))) is None


def test_no_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    with pytest.raises(RuntimeError):
        tlcgpu.Checker(tlcgpu.Model())


@pytest.mark.parametrize("keys", [2, 10, 15])
def test_jit_specialization_compiles(keys):
    """The hipRTC layout-specialized component kernels compile for gfx950
    without a device (a failure would silently fall back to the generic
    kernel at run time)."""
    m = tlcgpu.Model(key_space=range(1, keys + 1), value_space=range(1, keys + 1)).to_c()
    err = C.create_string_buffer(4096)
    n = tlcgpu.load_library().tlcg_jit_selftest(C.byref(m), b"gfx950", err, 4096)
    assert n > 0, err.value.decode()[:2000]


def test_wide_layouts_take_two_words():
    """> 63-bit layouts (CompactionTimesLimit = 12) are
    accepted as two-word states; the one-word entry points refuse them."""
    deep = tlcgpu.Model(compaction_times_limit=12, key_space=range(1, 11), value_space=range(1, 11))
    assert tlcgpu.check_model(deep) is None
    assert tlcgpu.state_bits(deep) > 63 and tlcgpu.state_words(deep) == 2
    assert tlcgpu.state_words(tlcgpu.Model()) == 1
    m = deep.to_c()
    lib = tlcgpu.load_library()
    assert lib.tlcg_decode(C.byref(m), 0, C.create_string_buffer(64), 64) < 0
    s0 = tlcgpu.host_init_state(deep, 5)
    assert "compactedLedgers = <<Nil, Nil, Nil, Nil, Nil, Nil, Nil, Nil, Nil, Nil, Nil, Nil>>" in tlcgpu.decode(deep, s0)
    succ = tlcgpu.host_successors(deep, s0)
    assert [a for a, _ in succ] == ["CompactorPhaseOne", "BrokerCrash"]
