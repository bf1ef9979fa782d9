"""Shared test fixtures.  `-m gpu` tests need an MI355X; everything else runs on CPU."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "pulsar-tlaplus_amd")
sys.path.insert(0, os.path.join(PKG, "python"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

LIB = os.path.join(PKG, "lib", "libtlcgpu.so")
CLI = os.path.join(PKG, "bin", "tlc-hip")
ORACLE = os.path.join(ROOT, "oracle", "build", "tlc_oracle")
REFERENCE = "/root/reference"

with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "golden.json")) as _f:
    GOLDEN = json.load(_f)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libtlcgpu.so on the device)")


def _ensure_built():
    if not os.path.exists(ORACLE):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, capture_output=True)
    if not os.path.exists(LIB) or not os.path.exists(CLI):
        subprocess.run(["make", "-C", PKG, "-j4"], check=True, capture_output=True)


@pytest.fixture(scope="session", autouse=True)
def built():
    _ensure_built()


def model_of(c):
    """tlcgpu.Model for a golden case's constants."""
    import tlcgpu
    return tlcgpu.Model(msg_sent_limit=c["N"], compaction_times_limit=c["C"], max_crash_times=c["K"],
                        consume_times_limit=c["ctl"], model_consumer=c["consumer"], model_producer=c["producer"],
                        retain_null_key=c["retain"], key_space=c["keys"], value_space=c["values"],
                        invariants=c["invariants"], check_deadlock=c["deadlock"])


def run_oracle(model, extra=()):
    out = subprocess.run([ORACLE] + model.oracle_args() + ["-levels"] + list(extra), check=True,
                         capture_output=True, text=True).stdout
    return json.loads(out)


FULL_CASES = sorted(k for k, v in GOLDEN.items() if "init_range" not in v["constants"])
