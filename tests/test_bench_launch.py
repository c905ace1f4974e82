"""bench.py --gpus N without a launcher: the plan it takes before anything
touches the GPU (relaunch under torch.distributed.run, run as one rank, or
refuse a --gpus that disagrees with the launcher's WORLD_SIZE)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_single_gpu_runs_in_process():
    assert bench.launch_plan(1, {}, []) == ("run", 1)


@pytest.mark.parametrize("n", [2, 4, 8])
def test_multi_gpu_without_launcher_relaunches(n):
    argv = ["--gpus", str(n), "--steps", "7", "--config", "glove"]
    kind, cmd = bench.launch_plan(n, {}, argv, port=29511)
    assert kind == "relaunch"
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert f"--nproc-per-node={n}" in cmd and "--nnodes=1" in cmd
    assert "--master-addr=127.0.0.1" in cmd and "--master-port=29511" in cmd
    i = cmd.index(os.path.join(ROOT, "bench.py"))
    assert cmd[i + 1:] == argv   # the same arguments reach every rank


def test_free_port_is_chosen():
    kind, cmd = bench.launch_plan(2, {}, [])
    port = int(next(a for a in cmd if a.startswith("--master-port=")).split("=")[1])
    assert 0 < port < 65536


def test_under_launcher_world_must_match():
    assert bench.launch_plan(8, {"WORLD_SIZE": "8"}, []) == ("run", 8)
    assert bench.launch_plan(1, {"WORLD_SIZE": "1"}, []) == ("run", 1)
    kind, msg = bench.launch_plan(1, {"WORLD_SIZE": "8"}, [])
    assert kind == "error" and "WORLD_SIZE=8" in msg
    assert bench.launch_plan(0, {}, [])[0] == "error"


def test_peek_gpus_ignores_other_flags():
    assert bench._peek_gpus(["--steps", "3", "--gpus", "4", "--no-sweep"]) == 4
    assert bench._peek_gpus([]) == 1


def test_mismatch_exits_nonzero_before_gpu():
    env = dict(os.environ, WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2
    assert "WORLD_SIZE=3" in r.stderr
