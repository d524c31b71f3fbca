"""bench.py's multi-rank launcher on the CPU (VERDICT r2 "next" 1): ``python bench.py --gpus N``
outside a torchrun environment starts N ranks itself (torch.distributed.run as a child process),
and rank 0's one JSON line reports the world size the process group actually had. ``--dry-run``
replaces the training step by a gloo all-reduce so the launcher, the rank environment, the
barrier + max-over-ranks timing and the strong-scaling batch split run without a GPU."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args, timeout=180):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    env.pop("LOCAL_RANK", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=timeout)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    return p.returncode, lines, p.stderr


@pytest.mark.parametrize("n", [2, 4, 8])
def test_gpus_n_launches_n_ranks(n):
    rc, lines, err = _run("--gpus", str(n), "--dry-run", "--steps", "3", "--warmup", "1")
    assert rc == 0, err[-2000:]
    assert len(lines) == 1, lines  # rank 0 only
    out = json.loads(lines[0])
    assert out["n_gpus"] == n and out["steps"] == 3 and out["warmup"] == 1
    assert out["scaling"] == "weak" and out["config"]["global_batch"] == 128 * n
    assert out["config"]["backend"] == "gloo"


def test_global_batch_is_split_over_ranks():
    rc, lines, err = _run("--gpus", "4", "--dry-run", "--steps", "2", "--warmup", "0", "--global-batch", "128")
    assert rc == 0, err[-2000:]
    out = json.loads(lines[0])
    assert out["scaling"] == "strong" and out["n_gpus"] == 4
    assert out["config"]["per_gpu_batch"] == 32 and out["config"]["global_batch"] == 128
    assert out["config"]["bn"] == "sync"


def test_global_batch_must_divide():
    rc, lines, err = _run("--gpus", "3", "--dry-run", "--steps", "1", "--warmup", "0", "--global-batch", "128")
    assert rc != 0 and not lines
    assert "not divisible" in err


def test_single_process_dry_run():
    rc, lines, err = _run("--dry-run", "--steps", "2", "--warmup", "0")
    assert rc == 0, err[-2000:]
    assert json.loads(lines[0])["n_gpus"] == 1
