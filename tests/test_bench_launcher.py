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


def _fake_topology(root, gpus, cpus=1, hidden=0):
    """A KFD topology tree: `cpus` CPU agents (simd_count 0), then `gpus` GPU agents whose render
    nodes exist under root/dri, then `hidden` GPU agents of the host whose render nodes this
    process cannot open (a container's view of the other GPUs)."""
    (root / "dri").mkdir(parents=True)
    for i in range(cpus + gpus + hidden):
        d = root / str(i)
        d.mkdir(parents=True)
        simd = 0 if i < cpus else 1024
        minor = 128 + i
        (d / "properties").write_text(f"cpu_cores_count 8\nsimd_count {simd}\n"
                                      f"max_waves_per_simd 8\ndrm_render_minor {minor}\n")
        if cpus <= i < cpus + gpus:
            (root / "dri" / f"renderD{minor}").write_text("")
    return str(root)


def test_visible_gpu_count_from_topology(tmp_path):
    b = _bench()
    topo = _fake_topology(tmp_path / "nodes", gpus=8, cpus=2, hidden=3)
    dri = os.path.join(topo, "dri")
    # the 3 host GPUs without an openable render node are not counted
    assert b.visible_gpu_count({}, kfd=topo, dri=dri) == 8
    assert b.visible_gpu_count({"HIP_VISIBLE_DEVICES": "0,1,2"}, kfd=topo, dri=dri) == 3
    assert b.visible_gpu_count({"ROCR_VISIBLE_DEVICES": "4", "HIP_VISIBLE_DEVICES": "0"},
                               kfd=topo, dri=dri) == 1
    assert b.visible_gpu_count({"CUDA_VISIBLE_DEVICES": ""}, kfd=topo, dri=dri) == 8
    # "-1" hides every device; ids after an invalid one are ignored by the runtime
    assert b.visible_gpu_count({"HIP_VISIBLE_DEVICES": "-1"}, kfd=topo, dri=dri) == 0
    assert b.visible_gpu_count({"CUDA_VISIBLE_DEVICES": "0,-1,2"}, kfd=topo, dri=dri) == 1
    assert b.visible_gpu_count({}, kfd=str(tmp_path / "absent"), dri=dri) is None


# the launcher parent under test: every way torch could reach hipGetDeviceCount raises, so a
# launcher that initialises HIP fails the test
_NO_HIP = r"""
import runpy, sys, torch
def _boom(*a, **k):
    raise RuntimeError("launcher parent called the HIP runtime")
torch._C._cuda_getDeviceCount = _boom
torch.cuda.device_count = _boom
torch.cuda.is_available = _boom
torch.cuda.init = _boom
sys.argv = [sys.argv[1]] + sys.argv[2:]
runpy.run_path(sys.argv[0], run_name="__main__")
"""


def test_launcher_parent_never_calls_hip(tmp_path):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("DLADMM_BENCH_BACKEND", None)
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        env.pop(var, None)
    # too few GPUs in the topology: refused before any rank starts, without a HIP call
    env["DLADMM_KFD_TOPOLOGY"] = _fake_topology(tmp_path / "two", gpus=2)
    p = subprocess.run([sys.executable, "-c", _NO_HIP, BENCH, "--gpus", "3",
                        "--launch-selftest"], env=env, capture_output=True, text=True,
                       timeout=120)
    assert p.returncode == 2, p.stderr[-2000:]
    assert "only 2 GPU(s) visible" in p.stderr and "HIP runtime" not in p.stderr
    # enough GPUs: the three ranks start and report
    env["DLADMM_KFD_TOPOLOGY"] = _fake_topology(tmp_path / "four", gpus=4)
    p = subprocess.run([sys.executable, "-c", _NO_HIP, BENCH, "--gpus", "3",
                        "--launch-selftest"], env=env, capture_output=True, text=True,
                       timeout=180)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1 and json.loads(lines[0])["ranks"] == [0, 1, 2]


def test_granted_cores_rules(monkeypatch, tmp_path):
    """cpu_baseline's thread count: the cgroup quota when set, else OMP_NUM_THREADS, else the
    affinity -- never more than the affinity."""
    b = _bench()
    import builtins
    real_open = builtins.open

    def fake_open(content):
        def op(path, *a, **k):
            if str(path) == "/sys/fs/cgroup/cpu.max":
                if content is None:
                    raise OSError("no cgroup")
                p = tmp_path / "cpu.max"
                p.write_text(content)
                return real_open(p, *a, **k)
            return real_open(path, *a, **k)
        return op

    aff = len(os.sched_getaffinity(0))
    monkeypatch.setattr(builtins, "open", fake_open("200000 100000\n"))
    monkeypatch.delenv("OMP_NUM_THREADS", raising=False)
    c, how = b.granted_cores()
    assert c == min(2, aff) and how["rule"] == "cgroup cpu.max quota"
    monkeypatch.setattr(builtins, "open", fake_open("max 100000\n"))
    monkeypatch.setenv("OMP_NUM_THREADS", "1")
    c, how = b.granted_cores()
    assert c == 1 and how["rule"].startswith("OMP_NUM_THREADS")
    monkeypatch.setattr(builtins, "open", fake_open(None))
    monkeypatch.delenv("OMP_NUM_THREADS", raising=False)
    c, how = b.granted_cores()
    assert c == aff and how["cgroup_cpu_max"] is None
