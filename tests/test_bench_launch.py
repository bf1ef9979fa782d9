"""bench.py --gpus N: the rank launcher (CPU; no torch, no GPU in the parent).

The driver runs `python bench.py --gpus N` for BENCH and `torch.distributed.run
--nproc-per-node N bench.py --gpus N` for SCALE; both must measure N ranks
(VERDICT r4 item 1)."""
import importlib.util
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load_bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_launch_plan():
    b = load_bench()
    assert b.launch_plan(1, {}) == ("run", None)
    assert b.launch_plan(8, {}) == ("spawn", 8)
    assert b.launch_plan(4, {"WORLD_SIZE": "4"}) == ("run", None)
    plan, why = b.launch_plan(8, {"WORLD_SIZE": "1"})
    assert plan == "refuse" and "WORLD_SIZE=1" in why
    assert b.launch_plan(0, {})[0] == "refuse"


CHILD = r"""
import json, os, sys
r, n = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
assert os.environ["LOCAL_RANK"] == str(r) and os.environ["MASTER_ADDR"] == "127.0.0.1"
assert int(os.environ["MASTER_PORT"]) > 0
print(json.dumps({"rank": r, "world": n}), flush=True)
if str(r) == os.environ.get("HANG_RANK"):
    import time
    time.sleep(600)
sys.exit(int(os.environ.get("FAIL_RANK_RC", "0")) if str(r) == os.environ.get("FAIL_RANK") else 0)
"""


def run_spawn(n, extra_env, grace=5.0):
    code = ("import importlib.util,sys;"
            f"s=importlib.util.spec_from_file_location('b',{os.path.join(ROOT, 'bench.py')!r});"
            "m=importlib.util.module_from_spec(s);s.loader.exec_module(m);"
            f"sys.exit(m.spawn_ranks({n},[sys.executable,'-c',{CHILD!r}],grace_s={grace}))")
    env = dict(os.environ, **extra_env)
    env.pop("WORLD_SIZE", None)
    return subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)


def test_spawn_ranks_rank0_stdout_only():
    p = run_spawn(3, {})
    assert p.returncode == 0, p.stderr
    lines = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")]
    assert lines == [{"rank": 0, "world": 3}]  # the other ranks' stdout went to stderr
    assert '"rank": 1' in p.stderr and '"rank": 2' in p.stderr


def test_spawn_ranks_failing_rank_sets_the_exit_code():
    p = run_spawn(2, {"FAIL_RANK": "1", "FAIL_RANK_RC": "7"})
    assert p.returncode == 7
    assert "rank 1 of 2 failed first (exit 7)" in p.stderr


def test_bench_refuses_a_mismatched_world():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 2 and "refused" in p.stderr and "WORLD_SIZE=2" in p.stderr


def test_spawn_ranks_ends_a_rank_left_hanging():
    """rank 1 fails, rank 0 waits in a 'collective' forever: terminated after the grace"""
    import time
    t = time.time()
    p = run_spawn(2, {"FAIL_RANK": "1", "FAIL_RANK_RC": "5", "HANG_RANK": "0"}, grace=2.0)
    assert p.returncode == 5
    assert time.time() - t < 60
