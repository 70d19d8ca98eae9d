"""Multi-GPU sharding of independent observation sequences (one process per GPU).

Sequences are independent, so a batch shards with no data-path collective: every rank holds the
(small) HMM, runs its share, and results are gathered once at the end.  Assignment is LPT
(longest processing time first, greedy onto the least-loaded rank) on sequence length, which
bounds the makespan by the longest sequence plus one average share.
"""
from __future__ import annotations

import heapq

import numpy as np


def lpt_assign(lengths, world_size: int) -> list[list[int]]:
    """Sequence indices per rank; longest first onto the least-loaded rank (ties: lower rank)."""
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


def gather_scores(local_idx, local_scores: np.ndarray, nseq: int, n: int, group=None, device=None):
    """Gather per-rank score rows to rank 0 in global sequence order (torch.distributed).

    One gather of a padded [max_local, n] tensor plus the index lists; works over gloo (CPU
    tensors) and nccl/RCCL (device tensors; pass `device`).  Returns the [nseq, n] array on rank
    0 and None elsewhere.
    """
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    counts = [None] * world
    dist.all_gather_object(counts, len(local_idx), group=group)
    width = max(max(counts), 1)
    buf = torch.full((width, n), float("inf"), dtype=torch.float32, device=device)
    if len(local_idx):
        buf[: len(local_idx)] = torch.as_tensor(np.asarray(local_scores, np.float32), device=device)
    gathered = [torch.empty_like(buf) for _ in range(world)] if rank == 0 else None
    if device is not None and str(device).startswith("cuda"):
        # RCCL has no gather; all_gather moves the same bytes for this tiny payload
        gathered = [torch.empty_like(buf) for _ in range(world)]
        dist.all_gather(gathered, buf, group=group)
    else:
        dist.gather(buf, gathered, dst=0, group=group)
    idx_lists = [None] * world
    dist.all_gather_object(idx_lists, list(map(int, local_idx)), group=group)
    if rank != 0:
        return None
    out = np.full((nseq, n), np.inf, np.float32)
    for r in range(world):
        rows = gathered[r].cpu().numpy()
        for k, q in enumerate(idx_lists[r]):
            out[q] = rows[k]
    return out
