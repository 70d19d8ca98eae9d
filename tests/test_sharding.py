"""Multi-rank sharding on CPU: LPT assignment and the gather of scores, best
states and decoded paths over gloo, world_size 2 and 3.

The shard compute is injected: the oracle (GraphBLAS_impl restatement) stands in for the GPU so
the distribution logic runs here; the GPU path of the same runner is covered in
tests/test_gpu_parity.py (world_size 1, HIP DeviceModel).
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from tests.conftest import chmm, ess
from tests.helpers import bit_equal

import spec_viterbi_amd as svh
from spec_viterbi_amd.sharding import lpt_assign


def test_lpt_assign_balances_and_covers():
    rng = np.random.default_rng(0)
    lengths = rng.integers(1, 7000, size=37)
    for world in (1, 2, 3, 8):
        parts = lpt_assign(lengths, world)
        flat = sorted(q for p in parts for q in p)
        assert flat == list(range(len(lengths)))
        loads = [int(sum(lengths[q] for q in p)) for p in parts]
        # LPT bound: makespan <= average share + longest job
        assert max(loads) <= sum(loads) / world + max(lengths)
        assert parts == lpt_assign(lengths, world)  # deterministic


def test_lpt_assign_covid_lengths():
    seqs = svh.read_emit_seq(ess("covid-19.ess"))
    lengths = [s.size for s in seqs]
    parts = lpt_assign(lengths, 8)
    loads = sorted(int(sum(lengths[q] for q in p)) for p in parts)
    assert loads[-1] == max(lengths)  # the longest sequence alone bounds the makespan
    assert sum(loads) == sum(lengths)


def test_lpt_more_ranks_than_sequences():
    parts = lpt_assign([5, 3], 4)
    assert sorted(map(len, parts)) == [0, 0, 1, 1]


def _oracle_compute(hmm, seqs, level, paths):
    from oracle import oracle

    if paths:
        out = [oracle.decode(hmm, s) for s in seqs]
        return (np.stack([o[0] for o in out]), np.array([o[1] for o in out], np.int64), [o[2] for o in out])
    scores = np.stack([oracle.viterbi(hmm, s) for s in seqs])
    best = np.array([int(np.argmin(r)) if np.isfinite(r).any() else -1 for r in scores], np.int64)
    return scores, best


def _worker(rank, world, port, model, ess_name, nseq, maxlen, paths, q):
    import torch.distributed as dist

    from spec_viterbi_amd.sharding import run_sharded

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        hmm = svh.read_HMM(chmm(model))
        seqs = [s[: maxlen - 97 * k] for k, s in enumerate(svh.read_emit_seq(ess(ess_name))[:nseq])]
        scores, best, pth, secs = run_sharded(hmm, seqs, paths=paths, compute=_oracle_compute)
        if rank == 0:
            q.put((scores, best, pth, secs))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world,paths", [(2, False), (2, True), (3, True)])
def test_run_sharded_gloo_matches_single_rank(world, paths):
    model, ess_name, nseq, maxlen = "100.chmm", "emit_3_3500_20.ess", 3, 400
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, model, ess_name, nseq, maxlen, paths, q))
             for r in range(world)]
    for p in procs:
        p.start()
    scores, best, pth, secs = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    hmm = svh.read_HMM(chmm(model))
    seqs = [s[: maxlen - 97 * k] for k, s in enumerate(svh.read_emit_seq(ess(ess_name))[:nseq])]
    ref = _oracle_compute(hmm, seqs, 0, paths)
    assert scores.shape == (nseq, hmm.states_num)
    for k in range(nseq):
        assert bit_equal(scores[k], ref[0][k])
    assert np.array_equal(best, ref[1])
    if paths:
        assert len(pth) == nseq
        for k in range(nseq):
            assert np.array_equal(pth[k], ref[2][k])
    assert secs >= 0
