"""bench.py's multi-GPU launch contract on the CPU.

`bench.py --gpus N` with no rank environment starts N ranks itself (a torch.distributed.run
child process), forwards rank 0's JSON line and exits with the children's status; under a
launcher WORLD_SIZE must equal --gpus.  `--dry-run` runs the same launch / gloo rendezvous /
max-over-ranks path with no GPU and no model."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
RANK_VARS = ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "LOCAL_WORLD_SIZE",
             "GROUP_RANK", "TORCHELASTIC_RUN_ID")


def _env(**extra):
    env = {k: v for k, v in os.environ.items() if k not in RANK_VARS}
    env.update(extra)
    env["OMP_NUM_THREADS"] = "1"
    return env


def _bench(args, env, timeout=240):
    return subprocess.run([sys.executable, str(ROOT / "bench.py")] + args, env=env, cwd=ROOT,
                          capture_output=True, text=True, timeout=timeout)


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _json_line(stdout):
    lines = [ln for ln in stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, f"expected exactly one JSON line (rank 0's), got {stdout!r}"
    return json.loads(lines[0])


@pytest.mark.parametrize("n", [1, 2])
def test_gpus_n_launches_n_ranks(n):
    p = _bench(["--gpus", str(n), "--dry-run", "--steps", "3", "--warmup", "1"], _env())
    assert p.returncode == 0, p.stderr[-2000:]
    line = _json_line(p.stdout)
    assert line["n_gpus"] == n
    assert sorted(r["rank"] for r in line["ranks"]) == list(range(n))
    assert sorted(r["local_rank"] for r in line["ranks"]) == list(range(n))
    assert line["steps"] == 3 and line["warmup"] == 1


def test_world_size_mismatch_is_refused():
    p = _bench(["--gpus", "2", "--dry-run"], _env(WORLD_SIZE="3", RANK="0", LOCAL_RANK="0"))
    assert p.returncode == 2
    assert "WORLD_SIZE=3" in p.stderr
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]


def test_launcher_matching_world_size_accepted():
    """The driver's form: torch.distributed.run sets WORLD_SIZE = --gpus itself."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", str(ROOT / "bench.py"),
           "--gpus", "2", "--dry-run", "--layout", "replicas"]
    p = subprocess.run(cmd, env=_env(), cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-2000:]
    line = _json_line(p.stdout)
    assert line["n_gpus"] == 2 and line["layout"] == "replicas"


def test_child_failure_propagates():
    """A rank that fails makes the launcher exit non-zero (no silent one-GPU result)."""
    p = _bench(["--gpus", "2", "--dry-run", "--steps", "-1"], _env())
    assert p.returncode != 0
