"""bench.py's N-rank launcher: `python bench.py --gpus N` must run N ranks, and a
WORLD_SIZE that disagrees with --gpus must fail loudly.  CPU only: the launch plan is host logic,
and `--launch-selftest` runs the real torch.distributed.run spawn with gloo ranks that never touch
a device."""
import importlib.util
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", BENCH)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_launch_plan_n_ranks():
    b = _bench()
    cmd, env = b.launch_plan(["--gpus", "8", "--steps", "5"], 8, 29511)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd
    assert "--master-addr=127.0.0.1" in cmd and "--master-port=29511" in cmd
    assert cmd[-3:] == ["--gpus", "8", "--steps", "5"][-3:]
    assert os.path.abspath(cmd[cmd.index(BENCH)]) == BENCH
    assert "WORLD_SIZE" not in env
    assert env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def test_world_check():
    b = _bench()
    assert b.world_check(1, {}) is None
    assert b.world_check(4, {}) == "launch"
    assert b.world_check(4, {"WORLD_SIZE": "4"}) is None
    with pytest.raises(SystemExit):
        b.world_check(8, {"WORLD_SIZE": "1"})
    with pytest.raises(SystemExit):
        b.world_check(1, {"WORLD_SIZE": "2"})
    with pytest.raises(SystemExit):
        b.world_check(0, {})


def test_world_size_mismatch_exits_nonzero():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, BENCH, "--gpus", "1"], env=env, capture_output=True,
                       text=True, timeout=120)
    assert p.returncode != 0
    assert "WORLD_SIZE=2" in p.stderr
    assert p.stdout.strip() == ""


def test_self_launch_spawns_n_gloo_ranks():
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, BENCH, "--gpus", "3", "--launch-selftest"], env=env,
                       capture_output=True, text=True, timeout=180)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout
    r = json.loads(lines[0])
    assert r["n_gpus"] == 3 and r["rank_sum"] == 3.0 and r["ranks"] == [0, 1, 2]
