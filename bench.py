#!/usr/bin/env python3
"""Headline benchmark: M state-updates/s (states x observations / s) of the Viterbi hot path on
2405.chmm x emit_50_3500_20.ess (BASELINE.json configs[2]), 1..N MI355X, weak scaling.

One step = one pass of the fused (min,+) Viterbi kernel over the whole batch (50 sequences x
3500 observations x 2407 states = 421,225,000 state-updates per GPU), inputs resident in HBM.
Multi-GPU: one process per GPU (torchrun); every rank runs its own 50-sequence batch (rank 0 the
reference file, rank r>0 same-shape synthetic sequences), no data-path collective; the timed
region is bracketed by barrier + synchronize and the max over ranks is reported.

Prints ONE JSON line (rank 0).  Extra fields: roofline (dominant kernel, HIP-event timed on the
stream it runs on) and cpu_baseline (the oracle, on this host's cores, bounded sample).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
DATA = os.path.join(ROOT, "data")

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
KERNEL_NAMES = {1: "fused", 2: "generic", 3: "band", 4: "chain"}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--level", type=int, default=0, help="0 = non-spec (headline); >=2 = _spec path")
    p.add_argument("--model", default="2405.chmm")
    p.add_argument("--ess", default="emit_50_3500_20.ess")
    p.add_argument("--kernel", type=int, default=0, help="0 auto, 1 fused, 2 generic")
    p.add_argument("--max-threads", type=int, default=0)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    p.add_argument("--no-check", action="store_true", help="skip the golden check (diagnostic ablations only)")
    p.add_argument("--paths", action="store_true", help="also decode paths (backpointers + traceback) every step")
    p.add_argument("--replicate", type=int, default=1,
                   help="batch = the file's sequences plus R-1 same-shape synthetic copies per GPU (full-chip "
                        "weak scaling, SURVEY 8(e): emit_50 x 8k sequences = --replicate 160); 1 = the headline")
    return p.parse_args()


def algorithmic_bytes_per_step(n: int, nnz: int) -> int:
    """streamed-CSR bytes of one observation of one sequence:
    8*nnz (value + index) + 4*(n+1) (row pointers) + 4n (emission row) + 4n (read v) + 4n (write v)."""
    return 8 * nnz + 4 * (n + 1) + 12 * n


def algorithmic_bytes_per_launch(n: int, nnz: int, lengths, level: int, paths: bool) -> int:
    """Bytes one launch must move under SURVEY.md 8(d)'s model, per sequence of length L:
    level <= 1: (L-1) streamed-CSR steps (+ 2n uint16 backpointers per step and 4 B per path entry
    with paths); level >= 2: floor((L-1)/level) dense products (4*n*round_up(n,4) + 8n each, the
    product is read whole) plus the (L-1) % level tail steps streamed-CSR."""
    step = algorithmic_bytes_per_step(n, nnz)
    total = 0
    for L in lengths:
        if level >= 2:
            chunks, tail = divmod(L - 1, level)
            total += chunks * (4 * n * ((n + 3) // 4 * 4) + 8 * n) + tail * step
        else:
            total += (L - 1) * step
            if paths:
                total += (L - 1) * 2 * n * 2 + 4 * L  # backpointers written and read back, path
    return total


def cpu_baseline(hmm, seqs, seconds: float) -> dict:
    """The oracle (C restatement of GraphBLAS_impl, -O2, OpenMP over sequences) on this host."""
    from oracle import oracle

    n = hmm.states_num
    threads = min(16, os.cpu_count() or 1)
    work = n * sum(int(s.size) for s in seqs)
    # multi-threaded passes over the whole batch, repeated for ~`seconds`
    times = []
    t_end = time.perf_counter() + seconds
    used = 1
    while time.perf_counter() < t_end or not times:
        t0 = time.perf_counter()
        _, used = oracle.viterbi_batch(hmm, seqs, nthreads=threads)
        times.append(time.perf_counter() - t0)
    med = float(np.median(times))
    # single-thread rate on a 4-sequence sample
    sample = seqs[:4]
    t0 = time.perf_counter()
    oracle.viterbi_batch(hmm, sample, nthreads=1)
    t1 = time.perf_counter() - t0
    single = n * sum(int(s.size) for s in sample) / t1 / 1e6
    return {
        "value": round(work / med / 1e6, 2), "unit": "M state-updates/s", "cores": int(used), "kind": "port",
        "sample": f"oracle/viterbi_oracle.c (GraphBLAS_impl restatement) over the full {len(seqs)}-sequence "
                  f"batch, median of {len(times)} passes on {used} OpenMP threads; 1 thread: {single:.1f} M/s "
                  f"on 4 sequences; host {os.cpu_count()} CPUs visible",
    }


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl", init_method="env://")
    torch.cuda.set_device(local)

    import spec_viterbi_amd as svh

    hmm = svh.read_HMM(os.path.join(DATA, "chmm_files", args.model))
    file_seqs = svh.read_emit_seq(os.path.join(DATA, "ess_files", args.ess))
    if rank == 0:
        seqs = file_seqs
    else:  # same-shape synthetic batch per extra rank (weak scaling)
        rng = np.random.default_rng(rank)
        seqs = [rng.integers(0, hmm.emit_num, size=s.size).astype(np.uint64) for s in file_seqs]
    if args.replicate > 1:
        rng = np.random.default_rng(1000 + rank)
        seqs = list(seqs) + [rng.integers(0, hmm.emit_num, size=s.size).astype(np.uint64)
                             for _ in range(args.replicate - 1) for s in file_seqs]
    n = int(hmm.states_num)
    model = svh.DeviceModel(hmm, device=local, kernel=args.kernel, max_threads=args.max_threads)
    info = model.info()
    prep_s = None
    if args.level >= 2:  # spec_with, timed apart from the run as bench_Viterbi_spec.h:69-71 does
        torch.cuda.synchronize()
        t_prep = time.perf_counter()
        model.spec_build(args.level)
        torch.cuda.synchronize()
        prep_s = time.perf_counter() - t_prep
    batch = model.batch(seqs, paths=args.paths)
    # A stream of our own: torch's default stream has handle 0, which the C ABI reads as "the
    # model's own stream", so events recorded on torch's default stream would not bracket the
    # kernel.  Every launch and every event below goes to this one stream.
    stream = torch.cuda.Stream(device=local)
    sptr = stream.cuda_stream
    assert sptr, "expected a non-null HIP stream handle"

    for _ in range(args.warmup):
        batch.run(args.level, sptr)
    torch.cuda.synchronize()

    starts = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    stops = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        starts[k].record(stream)
        batch.run(args.level, sptr)
        stops[k].record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kernel_ms = float(np.mean([s.elapsed_time(e) for s, e in zip(starts, stops)]))

    t = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{local}")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())

    # correctness guard on the timed output (rank 0 vs the committed golden of sequences 0..1)
    if (rank == 0 and not args.no_check and args.level <= 1 and args.model == "2405.chmm"
            and args.ess == "emit_50_3500_20.ess"):
        from tests.helpers import bit_equal, from_hex, load_golden

        scores, _ = batch.read(sptr)
        g = load_golden("chmm2405_emit50")
        for rec in g["sequences"]:
            assert bit_equal(scores[rec["index"]], from_hex(rec["scores"])), "bench output != golden"

    updates_per_rank = n * sum(int(s.size) for s in seqs)
    total_updates = updates_per_rank * world
    value = total_updates * args.steps / elapsed / 1e6
    ms_per_step = elapsed / args.steps * 1e3

    if rank == 0:
        nnz = int(info["nnz"])
        steps_obs = sum(int(s.size) for s in seqs)
        algo = algorithmic_bytes_per_launch(n, nnz, [int(x.size) for x in seqs], args.level, args.paths)
        achieved = algo / (kernel_ms * 1e-3) / 1e9
        traffic = None
        pmc_path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
        if os.path.exists(pmc_path) and args.level <= 1:
            with open(pmc_path) as f:
                traffic = json.load(f).get("hbm_bytes_per_launch")
        out = {
            "metric": f"M state-updates/sec (states x obs/s) on {args.model} x {args.ess}",
            "value": round(value, 2),
            "unit": "M state-updates/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "2405.chmm + emit_50_3500_20.ess (reference files) on rank 0; same-shape synthetic "
                    "sequences (numpy default_rng(rank)) on ranks > 0",
            "config": {
                "workload": f"{args.model} x {args.ess}" +
                            (f" x{args.replicate} (file sequences + same-shape synthetic copies)" if args.replicate > 1 else "") +
                            ", " + (f"non-spec (min,+) step, {KERNEL_NAMES.get(info['kernel'], '?')} kernel" if args.level <= 1
                                                              else f"_spec level {args.level}"),
                "states": n, "nnz": nnz, "sequences_per_gpu": len(seqs), "observations_per_gpu": steps_obs,
                "state_updates_per_gpu": updates_per_rank, "level": args.level,
                "kernel": (KERNEL_NAMES.get(info["paths_kernel"], "?") + "+traceback" if args.paths
                           else KERNEL_NAMES.get(info["kernel"], "?")),
                "paths": bool(args.paths), "spec_prep_s": None if prep_s is None else round(prep_s, 4), "threads": info["threads"],
                "slots": info["slots"], "heavy_rows": info["heavy_rows"], "heavy_uniform": info["heavy_uniform"],
                "parallelism": f"sequence-sharded x{world} (one process per GPU, no collective)",
            },
            "roofline": {
                "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                "kernel_ms": round(kernel_ms, 4),
                "note": "achieved = SURVEY 8(d) algorithmic bytes (47.98 B/state-update streamed-CSR model) / "
                        "HIP-event kernel time; the kernel keeps T^T in VGPRs and v in LDS, so it is on-chip "
                        "latency bound and frac > 1 is expected; traffic = PMC HBM bytes per launch",
            },
        }
        if not args.no_cpu_baseline and world == 1:
            out["cpu_baseline"] = cpu_baseline(hmm, file_seqs, args.cpu_seconds)
        print(json.dumps(out), flush=True)
    batch.close()
    model.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
