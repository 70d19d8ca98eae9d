"""CPU: bench.py's multi-process scaffolding (torchrun relaunch, WORLD_SIZE check, barriers,
max-over-ranks timing) with --dry-run over gloo; no GPU is touched."""
import json
import os
import subprocess
import sys

import pytest

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


@pytest.mark.parametrize("shard,nseq", [("emit50", 50), ("covid", 16)])
def test_gpus_2_strong_scaling_gathers_every_row(shard, nseq):
    """--shard emit50 / covid at N=2 over gloo: LPT shares of the real file, the post-timing gather
    of score rows and best states, every row placed at its global index on rank 0."""
    r = run("--gpus", "2", "--dry-run", "--shard", shard, "--steps", "2", "--warmup", "0")
    assert r.returncode == 0, r.stderr[-2000:]
    out = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")][-1]
    assert out["scaling"] == "strong" and out["sequences"] == nseq and sum(out["shares"]) == nseq
    assert min(out["shares"]) > 0 and out["gathered_ok"] is True


def test_gpus_2_failed_check_on_rank_1_fails_every_rank():
    """A rank whose timed output fails its check makes the whole job exit non-zero (rank 0 prints
    no result line)."""
    r = run("--gpus", "2", "--dry-run", "--dry-run-fail-rank", "1", "--steps", "2", "--warmup", "0")
    assert r.returncode != 0
    assert not [x for x in r.stdout.splitlines() if x.startswith("{")]


def test_digests_agree_with_goldens_and_catch_a_flipped_bit():
    """The committed digests bench.py checks against reproduce the golden rows 0..1 of
    2405 x emit_50 (independently stored as float bit patterns), and one flipped bit in a row is
    caught."""
    import numpy as np

    sys.path.insert(0, ROOT)
    import bench
    from tests.helpers import from_hex, load_golden

    ref = bench.digest_rows("2405.chmm", "emit_50_3500_20.ess")
    assert len(ref) == 50 and len(bench.digest_rows("2405.chmm", "covid-19.ess")) == 16
    g = load_golden("chmm2405_emit50")["sequences"]
    rows = np.stack([from_hex(r["scores"]) for r in g])
    best = np.array([r["best_state"] for r in g])
    idx = [r["index"] for r in g]
    assert bench.check_rows(rows, best, idx, ref) == []
    rows.view(np.uint32)[1, 7] ^= 1
    assert bench.check_rows(rows, best, idx, ref) == [idx[1]]
