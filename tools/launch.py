#!/usr/bin/env python3
"""Minimal launcher of the Viterbi step kernel for rocprofv3 passes (no torch import).

Builds one DeviceModel + DeviceBatch (the file's sequences plus R-1 same-shape synthetic copies,
as bench.py --replicate does), runs W untimed passes and K timed passes on the model's stream and
prints one JSON line with the mean HIP-event time per pass.  Output is checked bit-exact against
the committed digests of all 50 rows of 2405.chmm x emit_50_3500_20 when that is the workload.

    python3 tools/launch.py [--model 2405.chmm] [--ess emit_50_3500_20.ess] [--replicate R]
                            [--steps K] [--warmup W] [--level L] [--paths] [--nseq N] [--maxlen M]
                            [--kernel auto|pipe|pipew|diag|chain]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import spec_viterbi_amd as svh  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--model", default="2405.chmm")
    p.add_argument("--ess", default="emit_50_3500_20.ess")
    p.add_argument("--replicate", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--level", type=int, default=0)
    p.add_argument("--paths", action="store_true")
    p.add_argument("--nseq", type=int, default=0, help="use the first NSEQ sequences (0: all)")
    p.add_argument("--maxlen", type=int, default=0, help="truncate every sequence to MAXLEN observations (0: as read)")
    p.add_argument("--kernel", default="auto", help="svh_model_opts.kernel: auto, pipe, pipew, diag, chain")
    a = p.parse_args()
    hmm = svh.read_HMM(os.path.join(ROOT, "data", "chmm_files", a.model))
    seqs = svh.read_emit_seq(os.path.join(ROOT, "data", "ess_files", a.ess))
    if a.replicate > 1:
        rng = np.random.default_rng(1000)
        seqs = list(seqs) + [rng.integers(0, hmm.emit_num, size=s.size).astype(np.uint64)
                             for _ in range(a.replicate - 1) for s in seqs]
    if a.nseq:
        seqs = list(seqs)[: a.nseq]
    if a.maxlen:
        seqs = [s[: a.maxlen] for s in seqs]
    kern = {"auto": svh._lib.SVH_KERNEL_AUTO, "pipe": svh._lib.SVH_KERNEL_PIPE, "pipew": svh._lib.SVH_KERNEL_PIPE_WIDE,
            "diag": svh._lib.SVH_KERNEL_DIAG, "chain": svh._lib.SVH_KERNEL_CHAIN}[a.kernel]
    model = svh.DeviceModel(hmm, device=0, kernel=kern)
    if a.level >= 2:
        model.spec_build(a.level)
    batch = model.batch(seqs, paths=a.paths)
    for _ in range(a.warmup):
        batch.run(a.level)
    times = []
    for _ in range(a.steps):
        batch.run(a.level)
        times.append(batch.elapsed_ms())
    scores, _ = batch.read()
    ok = None
    # (diagnostic ablations, SVH_*_DEBUG or SVH_LAUNCH_NOCHECK=1 for ablation builds, give wrong
    # results by design: not checked)
    diag = any(os.environ.get(k) for k in ("SVH_PIPE_DEBUG", "SVH_BAND_DEBUG", "SVH_LAUNCH_NOCHECK"))
    if a.model == "2405.chmm" and a.ess == "emit_50_3500_20.ess" and a.level <= 2 and not diag and not a.maxlen:
        import hashlib

        from tests.helpers import load_digests

        key = "2405.chmm x emit_50_3500_20.ess" + ("" if a.level <= 1 else f" level {a.level}")
        rows = load_digests()[key]
        ok = all(hashlib.sha256(np.ascontiguousarray(scores[q], np.float32).tobytes()).hexdigest()
                 == rows[q]["scores_sha256"] for q in range(min(len(rows), len(seqs))))
    info = model.info()
    print(json.dumps({"model": a.model, "ess": a.ess, "replicate": a.replicate, "nseq": len(seqs),
                      "observations": int(sum(int(s.size) for s in seqs)), "level": a.level,
                      "paths": a.paths, "kernel_ms_mean": float(np.mean(times)), "kernel_ms": times,
                      "golden_ok": ok, "info": info}), flush=True)
    if ok is False:
        raise SystemExit("launch.py: output != golden")
    batch.close()
    model.close()


if __name__ == "__main__":
    main()
