"""bench.py's --gpus contract: N ranks are launched by the script itself when no launcher
ran it, and a launcher's WORLD_SIZE must agree with --gpus (VERDICT r4 "next" #1)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_check_world_rules():
    assert bench.check_world(1, {}) == "run"
    assert bench.check_world(2, {}) == "launch"
    assert bench.check_world(8, {"WORLD_SIZE": "8"}) == "run"
    assert bench.check_world(1, {"WORLD_SIZE": "1"}) == "run"
    with pytest.raises(SystemExit):
        bench.check_world(1, {"WORLD_SIZE": "2"})  # the driver's launcher, --gpus left at 1
    with pytest.raises(SystemExit):
        bench.check_world(4, {"WORLD_SIZE": "2"})
    with pytest.raises(SystemExit):
        bench.check_world(0, {})


def test_launch_command():
    cmd = bench.launch_ranks(4, ["--gpus", "4", "--steps", "3"])
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "127.0.0.1" in cmd
    assert cmd[-5:] == [os.path.join(ROOT, "bench.py"), "--gpus", "4", "--steps", "3"]


def _run(args, extra_env=None, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(extra_env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], env=env, cwd=ROOT,
                          capture_output=True, text=True, timeout=timeout)


def test_gpus2_self_launches_two_ranks():
    """`python bench.py --gpus 2` (no launcher) runs two ranks: the line says n_gpus 2,
    and the MAX over ranks saw rank 1's value (gloo on this GPU-less host)."""
    r = _run(["--gpus", "2", "--dry-run", "--cpu-baseline", "off"], {"LLFE_BENCH_SHARE_GPU": "1"})
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["dry_run"] is True
    assert d["max_over_ranks_probe"] == 1.0
    assert d["config"]["parallelism"] == "replicas x2 (host-side shard, no collective)"
    assert d["config"]["global_batch"] == 1024


def test_world_size_mismatch_fails_before_gpu():
    r = _run(["--gpus", "1", "--dry-run"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "must agree" in r.stderr


def test_gpus_more_than_visible_fails():
    # (one GPU visible by the environment; with no readable kfd topology at all the parent
    # leaves the check to the ranks)
    r = _run(["--gpus", "64", "--dry-run"], {"HIP_VISIBLE_DEVICES": "0"})
    assert r.returncode != 0
    assert "GPUs are visible" in r.stderr


@pytest.mark.gpu
def test_gpus2_real_run_on_one_gpu():
    """The whole bench, self-launched at --gpus 2, both ranks sharing cuda:0 (the box has
    one GPU): one line, n_gpus 2, a value from both ranks' images."""
    r = _run(["--gpus", "2", "--batch", "16", "--steps", "2", "--warmup", "1", "--cpu-baseline", "off",
              "--per-class-steps", "0", "--e2e-host-steps", "0", "--e2e-png-steps", "0", "--e2e-jpeg-steps", "0"],
             {"LLFE_BENCH_SHARE_GPU": "1"}, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["value"] > 0
    assert d["config"]["global_batch"] == 32
    assert d["config"]["parallelism"].startswith("replicas x2")


def test_visible_gpus_from_kfd_topology_without_hip(tmp_path):
    """The launching parent counts GPUs from sysfs (no HIP runtime in the parent)."""
    nodes = tmp_path / "nodes"
    for i, simds in enumerate([0, 1024, 1024, 0, 1024]):  # 2 CPU nodes, 3 GPUs
        (nodes / str(i)).mkdir(parents=True)
        (nodes / str(i) / "properties").write_text(f"cpu_cores_count 8\nsimd_count {simds}\nmax_waves_per_simd 8\n")
    assert bench.visible_gpus(env={}, sysfs=str(nodes)) == 3
    assert bench.visible_gpus(env={"HIP_VISIBLE_DEVICES": "0,1"}, sysfs=str(nodes)) == 2
    assert bench.visible_gpus(env={}, sysfs=str(tmp_path / "absent")) == 0
