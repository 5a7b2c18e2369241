"""bench.py's launcher contract (CPU): `python bench.py --gpus N` must run N ranks or fail — never
measure one GPU and report it as the N-GPU number ("What's missing" 3)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_rank_launch_command_spawns_n_ranks_without_launcher():
    cmd = bench.rank_launch_command(4, ["--gpus", "4", "--steps", "3"], {})
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "127.0.0.1" in cmd
    assert cmd[-4:] == ["--gpus", "4", "--steps", "3"]
    assert cmd[-5].endswith("bench.py")
    # already a rank (the driver's torch.distributed.run), or one GPU: run in this process
    assert bench.rank_launch_command(4, [], {"WORLD_SIZE": "4"}) is None
    assert bench.rank_launch_command(1, [], {}) is None


def test_world_size_must_equal_gpus():
    assert bench.check_world(1, {}) == 1
    assert bench.check_world(8, {"WORLD_SIZE": "8"}) == 8
    with pytest.raises(SystemExit):
        bench.check_world(2, {"WORLD_SIZE": "1"})
    with pytest.raises(SystemExit):
        bench.check_world(1, {"WORLD_SIZE": "2"})


def test_gpus_2_without_launcher_never_reports_one_gpu():
    """no GPU here: the two spawned ranks fail, so the command fails — what it must not do is
    print a line with n_gpus 1"""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["MASTER_ADDR"] = "127.0.0.1"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1",
                        "--warmup", "0", "--no-cpu-baseline"], env=env, capture_output=True, text=True,
                       timeout=300)
    for line in r.stdout.splitlines():
        if line.startswith("{"):
            assert json.loads(line)["n_gpus"] == 2
    if not any(l.startswith("{") for l in r.stdout.splitlines()):
        assert r.returncode != 0
    assert "starting 2 ranks" in r.stderr
