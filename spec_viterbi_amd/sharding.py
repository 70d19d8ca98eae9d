"""Multi-GPU sharding of independent observation sequences (one process per GPU), SURVEY.md 8(e).

Sequences are independent, so a batch shards with no data-path collective: every rank holds the
(small) HMM, runs its share on its own GPU, and results are gathered once at the end (scores,
best final states and, optionally, decoded paths).  Assignment is LPT (longest processing time
first, greedy onto the least-loaded rank) on sequence length, which bounds the makespan by the
longest sequence plus one average share.

The gathers are `dist.gather` of padded fixed-width tensors to rank 0 (ncclGather-style: only
rank 0 receives; the LPT assignment is deterministic, so no rank needs to exchange index lists).
The payloads are tiny (covid-19.ess: 16 x 2407 fp32 scores + 15,616 path entries), so they are
latency-bound on xGMI.  The same code runs over gloo on CPU tensors (the CPU tests).
"""
from __future__ import annotations

import heapq
import os
import time

import numpy as np


def lpt_assign(lengths, world_size: int) -> list[list[int]]:
    """Sequence indices per rank; longest first onto the least-loaded rank (ties: lower rank)."""
    if world_size < 1:
        raise ValueError("world_size must be >= 1")
    order = sorted(range(len(lengths)), key=lambda q: (-int(lengths[q]), q))
    heap = [(0, r) for r in range(world_size)]
    heapq.heapify(heap)
    out: list[list[int]] = [[] for _ in range(world_size)]
    for q in order:
        load, r = heapq.heappop(heap)
        out[r].append(q)
        heapq.heappush(heap, (load + int(lengths[q]), r))
    for r in range(world_size):
        out[r].sort()
    return out


def _gather_rows(assignment, rows: np.ndarray, nseq: int, fill, group=None, device=None):
    """Gather per-rank rows [len(assignment[rank]), width] to rank 0, placed by global index.

    `assignment` is the full LPT assignment (deterministic, so every rank holds it): each rank
    pads its rows to the largest share and one `dist.gather` (RCCL gather on GPUs, gloo on
    CPUs) brings them to rank 0, which alone allocates the receive buffers.  Returns
    [nseq, width] on rank 0, None elsewhere.
    """
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    mine = assignment[rank]
    rows = np.asarray(rows)
    width = rows.shape[1] if rows.ndim == 2 else 1
    height = max(max(len(a) for a in assignment), 1)
    dtype = torch.from_numpy(np.zeros(0, rows.dtype)).dtype
    buf = torch.full((height, width), fill, dtype=dtype, device=device)
    if len(mine):
        buf[: len(mine)] = torch.from_numpy(np.ascontiguousarray(rows.reshape(len(mine), width))).to(buf.device)
    recv = [torch.empty_like(buf) for _ in range(world)] if rank == 0 else None
    dist.gather(buf, recv, dst=0, group=group)
    if rank != 0:
        return None
    out = np.full((nseq, width), fill, rows.dtype)
    for r in range(world):
        got = recv[r].cpu().numpy()
        for k, q in enumerate(assignment[r]):
            out[q] = got[k]
    return out


def gather_scores(assignment, local_scores: np.ndarray, nseq: int, n: int, group=None, device=None):
    """Per-rank score rows [len(assignment[rank]), n] -> [nseq, n] fp32 on rank 0 (None elsewhere)."""
    import torch.distributed as dist

    mine = assignment[dist.get_rank(group)]
    rows = np.asarray(local_scores, np.float32).reshape(len(mine), n)
    return _gather_rows(assignment, rows, nseq, float("inf"), group, device)


def gather_paths(assignment, local_paths, lengths, group=None, device=None):
    """Per-rank decoded paths (int32 arrays) -> list of nseq paths on rank 0 (None elsewhere)."""
    import torch.distributed as dist

    mine = assignment[dist.get_rank(group)]
    width = max([int(x) for x in lengths] + [1])
    rows = np.full((len(mine), width), -1, np.int32)
    for k, p in enumerate(local_paths):
        rows[k, : len(p)] = p
    out = _gather_rows(assignment, rows, len(lengths), -1, group, device)
    if out is None:
        return None
    return [out[q, : int(lengths[q])].copy() for q in range(len(lengths))]


def _hip_compute(device: int, time_parallel=None):
    """The product's shard compute: one DeviceModel batch on this rank's GPU (fails loudly
    without the HIP library).  time_parallel = (seg_len, probe_len): the opt-in time-parallel
    pass (scores only, level 0) -- a rank's makespan is otherwise its longest
    sequence."""
    from .viterbi import DeviceModel

    def compute(hmm, seqs, level: int, paths: bool):
        if time_parallel and (paths or level >= 2):
            raise ValueError("time-parallel runs compute scores only at level 0/1")
        model = DeviceModel(hmm, device=device)
        try:
            if level >= 2:
                model.spec_build(level)
            batch = model.batch(seqs, paths=paths)
            try:
                if time_parallel:
                    batch.run_time_parallel(seg_len=time_parallel[0], probe_len=time_parallel[1])
                else:
                    batch.run(level)
                return batch.read(want_paths=paths)
            finally:
                batch.close()
        finally:
            model.close()

    return compute


def run_sharded(hmm, seqs, *, level: int = 0, paths: bool = False, group=None, device=None,
                compute=None, time_parallel=None):
    """Viterbi over `seqs` sharded across the ranks of `group` (torch.distributed, initialised).

    Each rank runs its LPT share with `compute(hmm, local_seqs, level, paths)` -- by default the
    HIP DeviceModel on `device` (this rank's GPU) -- and the results are gathered to rank 0.
    `device` is also where the gather tensors live ("cuda:k" for RCCL, None for gloo).
    Returns (scores [nseq, n], best [nseq], paths or None, seconds_max_over_ranks) on rank 0 and
    (None, None, None, seconds) elsewhere.
    """
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    lengths = [int(np.asarray(s).size) for s in seqs]
    assignment = lpt_assign(lengths, world)
    mine = assignment[rank]
    if compute is None:
        index = torch.device(device).index if device is not None else int(os.environ.get("LOCAL_RANK", "0"))
        compute = _hip_compute(index or 0, time_parallel)
    n = int(hmm.states_num)
    dist.barrier(group)
    t0 = time.perf_counter()
    if mine:
        res = compute(hmm, [seqs[q] for q in mine], level, paths)
        scores, best = res[0], res[1]
        local_paths = res[2] if paths else []
    else:
        scores = np.zeros((0, n), np.float32)
        best = np.zeros(0, np.int64)
        local_paths = []
    seconds = time.perf_counter() - t0
    t = torch.tensor([seconds], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    seconds = float(t.item())
    all_scores = gather_scores(assignment, scores, len(seqs), n, group, device)
    all_best = _gather_rows(assignment, np.asarray(best, np.int64).reshape(-1, 1), len(seqs), -1, group, device)
    all_paths = gather_paths(assignment, local_paths, lengths, group, device) if paths else None
    if rank != 0:
        return None, None, None, seconds
    return all_scores, all_best.reshape(-1), all_paths, seconds
