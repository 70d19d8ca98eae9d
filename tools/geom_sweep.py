#!/usr/bin/env python3
"""Latency-plan geometry for few-sequence batches (the strong-scaling shares): for batches of the
first N sequences of a file, the pipelined latency plan's kernel time (HIP events, median of REPS)
in each geometry (slots per lane x waves per workgroup, SVH_PIPE_SM / SVH_PIPE_WAVES, read at
model creation), every result checked bit-exact against the first geometry's.

    python3 tools/geom_sweep.py [--ess covid-19.ess] [--counts 1,2,4,7,16] [--geoms 2x4,1x4,1x8,2x8]
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
from spec_viterbi_amd import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="2405.chmm")
    ap.add_argument("--ess", default="covid-19.ess")
    ap.add_argument("--counts", default="1,2,4,7,16")
    ap.add_argument("--geoms", default="2x4,1x4,1x8,2x8")
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    hmm = svh.read_HMM(os.path.join(ROOT, "data", "chmm_files", a.model))
    seqs = svh.read_emit_seq(os.path.join(ROOT, "data", "ess_files", a.ess))
    # longest first: the shares a rank gets from lpt_assign start with the longest rows
    seqs = sorted(seqs, key=lambda s: -s.size)
    out = {"model": a.model, "ess": a.ess, "rows": {}}
    for n in [int(c) for c in a.counts.split(",")]:
        batch_seqs = seqs[:n]
        ref = None
        row = {"observations": int(sum(s.size for s in batch_seqs))}
        for g in a.geoms.split(","):
            sm, w = g.split("x")
            os.environ["SVH_PIPE_SM"], os.environ["SVH_PIPE_WAVES"] = sm, w
            model = svh.DeviceModel(hmm, device=0, kernel=_lib.SVH_KERNEL_PIPE)
            b = model.batch(batch_seqs)
            ts = []
            for _ in range(a.reps + 1):
                b.run()
                ts.append(b.elapsed_ms())
            s, best = b.read()
            if ref is None:
                ref = (s, best)
            same = bool(np.array_equal(s.view(np.uint32), ref[0].view(np.uint32)) and np.array_equal(best, ref[1]))
            row[g] = {"ms": round(float(np.median(ts[1:])), 4), "same_as_first": same, "fallbacks": b.fallbacks(),
                      "groups": b.plan()["pipe_groups"]}
            b.close()
            model.close()
        out["rows"][n] = row
        print(json.dumps({n: row}), flush=True)
    del os.environ["SVH_PIPE_SM"], os.environ["SVH_PIPE_WAVES"]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
