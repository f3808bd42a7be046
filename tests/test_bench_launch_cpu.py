"""bench.py's launch contract on the CPU: `--gpus N` without a launcher
starts N ranks itself (torch.distributed.run as a child process) and never prints a silent
one-rank line; a launcher whose WORLD_SIZE disagrees with --gpus is an error."""
import json
import os
import subprocess
import sys

from conftest import REPO

BENCH = os.path.join(REPO, "bench.py")


def _run(args, env_extra=None, timeout=180):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                             "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True, timeout=timeout,
                          env=env, cwd=REPO)


def _json_lines(out):
    return [json.loads(l) for l in out.splitlines() if l.startswith("{")]


def test_gpus_n_spawns_n_ranks():
    r = _run(["--gpus", "2", "--dist-backend", "gloo", "--launch-selftest"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout  # rank 0 only
    assert lines[0]["n_gpus"] == 2 and lines[0]["ranks_seen"] == 2


def test_gpus_3_spawns_3_ranks():
    r = _run(["--gpus", "3", "--dist-backend", "gloo", "--launch-selftest"])
    assert r.returncode == 0, r.stderr[-2000:]
    assert _json_lines(r.stdout)[0]["n_gpus"] == 3


def test_world_size_disagreeing_with_gpus_fails():
    r = _run(["--gpus", "2", "--dist-backend", "gloo", "--launch-selftest"],
             {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert not _json_lines(r.stdout)
    assert "WORLD_SIZE 1" in r.stderr


def test_rccl_without_enough_gpus_fails_loudly():
    import torch
    if torch.cuda.device_count() >= 2:
        import pytest
        pytest.skip("two GPUs visible")
    r = _run(["--gpus", "2", "--launch-selftest"])
    assert r.returncode != 0
    assert not _json_lines(r.stdout)
    assert "needs 2 GPUs" in r.stderr


def test_launcher_without_gpus_takes_its_world_size():
    """(round-4 advisor) `torchrun --nproc-per-node N bench.py` without --gpus runs N ranks."""
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                        "--master-addr", "127.0.0.1", f"--master-port={port}", BENCH, "--dist-backend", "gloo",
                        "--launch-selftest"], capture_output=True, text=True, timeout=180, env=env, cwd=REPO)
    assert r.returncode == 0, r.stderr[-2000:]
    assert _json_lines(r.stdout)[0]["n_gpus"] == 2
