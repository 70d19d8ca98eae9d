"""CPU: bench.py's multi-process scaffolding (torchrun relaunch, WORLD_SIZE check, barriers,
max-over-ranks timing) with --dry-run over gloo; no GPU is touched."""
import json
import os
import subprocess
import sys

from tests.conftest import ROOT

BENCH = os.path.join(ROOT, "bench.py")


def run(*args, env=None):
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    e.update(env or {})
    return subprocess.run([sys.executable, BENCH, *args], capture_output=True, text=True, timeout=180, env=e)


def test_gpus_2_relaunches_two_ranks():
    r = run("--gpus", "2", "--dry-run", "--steps", "4", "--warmup", "1")
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 alone prints
    out = lines[0]
    assert out["n_gpus"] == 2 and out["steps"] == 4
    # max over ranks: rank 1 sleeps 2 ms per step
    assert out["ms_per_step"] >= 2.0


def test_gpus_1_runs_in_process():
    r = run("--gpus", "1", "--dry-run", "--steps", "3", "--warmup", "0")
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["n_gpus"] == 1


def test_world_size_mismatch_fails():
    r = run("--gpus", "4", "--dry-run", env={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr
