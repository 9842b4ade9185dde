"""bench.py's launch logic (CPU): `--gpus N` must really run N ranks.

`plan()` decides how an invocation runs; `--dry-run` sets the ranks up over gloo and
prints the plan without touching a GPU, so the child-torchrun path is exercised end to
end here."""
import argparse
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def _args(*a):
    return bench.parse(list(a))


def test_plan_modes():
    assert bench.plan(_args(), {}) == ("single", 1)
    assert bench.plan(_args("--gpus", "1"), {}) == ("single", 1)
    assert bench.plan(_args("--gpus", "8"), {}) == ("launch", 8)
    assert bench.plan(_args("--gpus", "8"), {"WORLD_SIZE": "8"}) == ("ranks", 8)
    assert bench.plan(_args("--gpus", "1"), {"WORLD_SIZE": "1"}) == ("ranks", 1)
    assert bench.plan(_args("--device-list", "0,1,2,3"), {}) == ("device-list", [0, 1, 2, 3])
    with pytest.raises(SystemExit):
        bench.plan(_args("--device-list", "0,1"), {"WORLD_SIZE": "2"})


def test_launch_command_shape():
    cmd = bench.launch_cmd(["--gpus", "4", "--steps", "3"], 4, 29555)
    assert cmd[1:4] == ["-m", "torch.distributed.run", "--nnodes=1"]
    assert "--nproc-per-node=4" in cmd and "127.0.0.1" in cmd and "--master-port=29555" in cmd
    assert cmd[-5].endswith("bench.py") and cmd[-4:] == ["--gpus", "4", "--steps", "3"]


def test_gpus_two_spawns_two_ranks():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run"],
                       cwd=ROOT, capture_output=True, text=True, timeout=170)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d == {"dry_run": True, "mode": "ranks", "world": 2, "ranks_seen": 2, "n_gpus": 2}


def test_gpus_beyond_visible_devices_fails_loudly(monkeypatch):
    """Never a silent n_gpus = 1 when more were asked for."""
    monkeypatch.setattr(bench, "visible_gpus", lambda env=None: 1)
    with pytest.raises(SystemExit, match="needs 4 visible GPUs"):
        bench.launch_ranks(["--gpus", "4"], 4, dry_run=False)


def test_visible_gpus_never_initialises_hip(monkeypatch):
    """the parent counts devices from the environment / KFD topology, not through
    hipGetDeviceCount (which would initialise HSA before the ranks start)."""
    def boom():
        raise AssertionError("HIP touched in the launching parent")
    monkeypatch.setattr(bench.torch.cuda, "device_count", boom)
    assert bench.visible_gpus({"HIP_VISIBLE_DEVICES": "0,1,2"}) == 3
    assert bench.visible_gpus({"ROCR_VISIBLE_DEVICES": "4"}) == 1
    n = bench.visible_gpus({})
    assert n is None or n >= 0


def test_host_cores_respects_quota(monkeypatch):
    monkeypatch.setattr(bench, "_cpu_quota", lambda: 16.0)
    monkeypatch.setattr(bench.os, "sched_getaffinity", lambda pid: set(range(256)))
    assert bench.host_cores() == (16, 256, 16.0)
    monkeypatch.setattr(bench, "_cpu_quota", lambda: None)
    assert bench.host_cores()[0] == 256


def test_bench_configs_gpus_two_spawns_two_ranks():
    """bench_configs.py --gpus N runs N ranks from one command (C3 over 8 GPUs)."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench_configs.py"), "--gpus", "2", "--dry-run",
                        "--only", "C3"], cwd=ROOT, capture_output=True, text=True, timeout=170)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    assert json.loads(lines[0]) == {"dry_run": True, "mode": "ranks", "world": 2, "ranks_seen": 2, "n_gpus": 2}


def test_parallelism_label_states_whether_rccl_ran():
    """The N = 1 line started directly has no process group: its label must not claim RCCL
    (VERDICT r5 #7); under torchrun (world 1 included) the counters go through RCCL."""
    single = bench.parallelism_label("single", 1, None, 10)
    assert "RCCL" not in single and "no collective" in single
    assert "RCCL" in bench.parallelism_label("ranks", 1, None, 10)
    assert "x8 ranks" in bench.parallelism_label("ranks", 8, None, 10)
    dl = bench.parallelism_label("device-list", 1, [0, 1], 10)
    assert "RCCL" not in dl and "[0, 1]" in dl


def test_pmc_profile_prefers_the_profile_of_this_build(monkeypatch, tmp_path):
    """A profile taken on the running libpsg.so wins over a later-named one of another build."""
    a = _args()
    w = {"n": a.n, "rounds": a.rounds, "instances_per_gpu": a.instances, "value_range": a.V}

    def put(name, sha):
        d = tmp_path / "profiles" / name
        d.mkdir(parents=True)
        (d / "pmc_summary.json").write_text(json.dumps(
            {"kernel": "psg::otr_kernel<1, false>", "hbm": {}, "per_instance_round": {}, "workload": w,
             "lib_sha256": sha}))

    put("r6_otr_n64", "this")
    put("r6m_otr_n64", "older")
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    monkeypatch.setattr(bench, "lib_sha256", lambda: "this")
    path, _, same = bench.pmc_profile(a)
    assert path == os.path.join("profiles", "r6_otr_n64", "pmc_summary.json") and same
    monkeypatch.setattr(bench, "lib_sha256", lambda: "another")
    path, _, same = bench.pmc_profile(a)
    assert path == os.path.join("profiles", "r6m_otr_n64", "pmc_summary.json") and not same
