"""CPU: the user-invariant compiler under AddressSanitizer and UBSan
(tests/fuzz/user_inv_fuzz.cpp, host code only: user_inv.cpp and
host_model.cpp built with g++ -fsanitize=address,undefined).  Every
definition of the user-invariant fixtures (tests/user_inv_cases.py, the bench
configs' invariants) is compiled as written and as deterministic mutations;
each compile must end in a program or a refusal with a message, each program
must generate device code and evaluate to TRUE / FALSE / error on every
reachable state of a small model, with no sanitizer report."""
import json
import os
import shutil
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, HERE)
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "pulsar-tlaplus_amd", "python"))

CSRC = os.path.join(ROOT, "pulsar-tlaplus_amd", "csrc")


def corpus_text():
    import tlcgpu as T
    from user_inv_cases import CASES, HELPERS
    from bench import USER_DEFS
    out = []
    for name, body in sorted(CASES.items()):
        m = T.Model(invariants=(name,), user_defs={**HELPERS, name: body})
        out.append(f"@@CASE {name}\n" + m.user_defs_text())
    for name in ("PhaseKnown", "LatestIsLast", "LedgerSorted", "KeysKnown", "MessageRec", "HeadFirst"):
        m = T.Model(invariants=(name,), user_defs=dict(USER_DEFS))
        out.append(f"@@CASE {name}\n" + m.user_defs_text())
    return "".join(out), len(CASES) + 6


@pytest.fixture(scope="module")
def fuzz_bin(tmp_path_factory):
    if shutil.which("g++") is None:
        pytest.skip("g++ not found")
    d = tmp_path_factory.mktemp("fuzz")
    exe = str(d / "user_inv_fuzz")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined",
           "-fno-omit-frame-pointer", "-I" + os.path.join(ROOT, "include"), "-I" + CSRC,
           os.path.join(HERE, "fuzz", "user_inv_fuzz.cpp"), os.path.join(CSRC, "host_model.cpp"),
           os.path.join(CSRC, "user_inv.cpp"), "-o", exe]
    subprocess.run(cmd, check=True, timeout=600)
    return exe


@pytest.mark.parametrize("seed", [1, 2])
def test_user_inv_compiler_under_sanitizers(fuzz_bin, tmp_path, seed):
    text, n = corpus_text()
    corpus = tmp_path / "corpus.txt"
    corpus.write_text(text)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([fuzz_bin, str(corpus), "60", str(seed)], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["entries"] == n and res["unmutated_ok"] == n  # every fixture compiles as written
    assert res["compiled"] > n and res["refused"] > 0 and res["evals"] > 0
    assert res["true"] + res["false"] + res["error"] == res["evals"]
    # the outcome tables agree with the programs (component_code.h code_consts_user)
    assert res["table_checks"] > 0 and res["static_checks"] > 0


REF = "/root/reference"


@pytest.fixture(scope="module")
def cfg_fuzz_bin(tmp_path_factory):
    if shutil.which("g++") is None:
        pytest.skip("g++ not found")
    d = tmp_path_factory.mktemp("cfgfuzz")
    exe = str(d / "cfg_fuzz")
    host = os.path.join(ROOT, "pulsar-tlaplus_amd", "host")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined",
           "-fno-omit-frame-pointer", "-I" + os.path.join(ROOT, "include"), "-I" + CSRC, "-I" + host,
           os.path.join(HERE, "fuzz", "cfg_fuzz.cpp"), os.path.join(host, "cfg.cpp"),
           os.path.join(CSRC, "host_model.cpp"), os.path.join(CSRC, "user_inv.cpp"), "-o", exe]
    subprocess.run(cmd, check=True, timeout=600)
    return exe


@pytest.mark.skipif(not os.path.exists(os.path.join(REF, "compaction.tla")), reason="reference spec absent")
def test_cli_front_end_under_sanitizers(cfg_fuzz_bin, tmp_path):
    """tlc-hip's cfg parser, module reader, recognition and constants binding
    (host/cfg.cpp) on the reference's compaction.tla and its cfg with numeric
    keys, as written and mutated: a result or a message with an exit code,
    no sanitizer report"""
    text = open(os.path.join(REF, "compaction.cfg")).read().replace('"key1", "key2"', "1, 2")
    cfg = tmp_path / "num.cfg"
    cfg.write_text(text)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([cfg_fuzz_bin, str(cfg), os.path.join(REF, "compaction.tla"), "200", "1"], capture_output=True,
                       text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["bound"] > 0 and res["refused"] > 0 and res["recognized"] > 0
