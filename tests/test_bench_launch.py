"""bench.py's N-rank launch: `bench.py --gpus N` without a
launcher starts torch.distributed.run with N ranks as a child process, and a
WORLD_SIZE that disagrees with --gpus is an error, not a silent one-rank run."""
from __future__ import annotations

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def _args(*argv):
    old = sys.argv
    sys.argv = ["bench.py", *argv]
    try:
        return bench.parse()
    finally:
        sys.argv = old


def test_one_gpu_runs_in_process():
    assert bench.check_launch(_args(), env={}) is None
    assert bench.check_launch(_args("--gpus", "1"), env={}) is None


def test_n_gpus_without_launcher_builds_torchrun_child():
    old = sys.argv
    sys.argv = ["bench.py", "--gpus", "4", "--steps", "7", "--exchange", "factored"]
    try:
        cmd = bench.check_launch(bench.parse(), env={})
    finally:
        sys.argv = old
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd and "--master-addr=127.0.0.1" in cmd
    i = cmd.index(os.path.join(ROOT, "bench.py"))
    assert cmd[i + 1:] == ["--gpus", "4", "--steps", "7", "--exchange", "factored"]


def test_under_launcher_world_size_must_match():
    assert bench.check_launch(_args("--gpus", "8"), env={"WORLD_SIZE": "8"}) is None
    with pytest.raises(SystemExit, match="WORLD_SIZE=8 but --gpus 1"):
        bench.check_launch(_args(), env={"WORLD_SIZE": "8"})
    with pytest.raises(SystemExit, match="WORLD_SIZE=2 but --gpus 4"):
        bench.check_launch(_args("--gpus", "4"), env={"WORLD_SIZE": "2"})
    with pytest.raises(SystemExit, match="must be >= 1"):
        bench.check_launch(_args("--gpus", "0"), env={})


def test_mismatch_exits_nonzero_before_any_work():
    env = dict(os.environ, WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert "WORLD_SIZE=3 but --gpus 2" in r.stderr
    assert not r.stdout.strip()


def test_rccl_launch_refuses_more_ranks_than_devices():
    # no GPU here: RCCL ranks cannot share one device, so N > visible devices is refused up front
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert "RCCL needs 2 devices" in r.stderr


def test_launcher_starts_n_ranks(tmp_path):
    """The real child launch (gloo, CPU): two ranks start, see WORLD_SIZE = 2
    and rank 0 prints the line."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-backend", "gloo",
                        "--launch-probe"], env=env, capture_output=True, text=True, timeout=300, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert lines == [{"n_gpus": 2, "rank_sum": 3}]
