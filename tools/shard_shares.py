#!/usr/bin/env python3
"""Strong-scaling forecast from one GPU: for N = 1, 2, 4, 8 ranks, the LPT share of every rank
(spec_viterbi_amd.sharding.lpt_assign, exactly what bench.py --shard uses) is timed on this GPU,
one share after another (HIP events, median of REPS passes, AUTO plan of that share's batch), and
the makespan is the slowest share.  Forecast speedup(N) = makespan(1) / makespan(N), compute only
(the RCCL gather after the timed region and the launch skew between ranks are not in it).
Every share's scores are checked against the committed digests.

    python3 tools/shard_shares.py [--shard covid|emit50] [--reps 10]
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import spec_viterbi_amd as svh  # noqa: E402
from spec_viterbi_amd.sharding import lpt_assign  # noqa: E402
from tests.helpers import load_digests  # noqa: E402

FILES = {"covid": "covid-19.ess", "emit50": "emit_50_3500_20.ess"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shard", default="covid", choices=sorted(FILES))
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--ranks", default="1,2,4,8")
    a = ap.parse_args()
    hmm = svh.read_HMM(os.path.join(ROOT, "data", "chmm_files", "2405.chmm"))
    seqs = svh.read_emit_seq(os.path.join(ROOT, "data", "ess_files", FILES[a.shard]))
    rows = load_digests()[f"2405.chmm x {FILES[a.shard]}"]
    model = svh.DeviceModel(hmm, device=0)
    out = {"shard": a.shard, "file": FILES[a.shard], "lengths": [int(s.size) for s in seqs], "ranks": {}}
    ok = True
    for world in [int(x) for x in a.ranks.split(",")]:
        assignment = lpt_assign([s.size for s in seqs], world)
        shares = []
        for r, idx in enumerate(assignment):
            if not idx:
                shares.append({"rank": r, "rows": [], "ms": 0.0})
                continue
            batch = model.batch([seqs[q] for q in idx])
            ts = []
            for _ in range(a.reps + 1):
                batch.run()
                ts.append(batch.elapsed_ms())
            scores, _ = batch.read()
            for k, q in enumerate(idx):
                ok &= hashlib.sha256(np.ascontiguousarray(scores[k], np.float32).tobytes()).hexdigest() == \
                    rows[q]["scores_sha256"]
            plan = batch.plan()
            shares.append({"rank": r, "rows": idx, "observations": int(sum(seqs[q].size for q in idx)),
                           "ms": round(float(np.median(ts[1:])), 4), "kernel": plan["kernel"],
                           "fallbacks": batch.fallbacks()})
            batch.close()
        mk = max(s["ms"] for s in shares)
        out["ranks"][world] = {"makespan_ms": mk, "shares": shares}
    base = out["ranks"].get(1, {}).get("makespan_ms")
    for world, v in out["ranks"].items():
        v["forecast_speedup"] = round(base / v["makespan_ms"], 3) if base else None
    out["digests_ok"] = bool(ok)
    print(json.dumps(out), flush=True)
    model.close()
    if not ok:
        raise SystemExit("shard_shares: a share's scores differ from the digests")


if __name__ == "__main__":
    main()
