#!/usr/bin/env python3
"""The reference harness's sweep on the MI355X backend: every .chmm x the four datasets of
main.cpp (emit_3_3500_20, emit_3_7000_20, covid-19, emit_50_3500_20; /root/reference main.cpp:5-6,
19-20), non-spec and _spec levels 1..2 (bench_Viterbi.h:37-48, bench_Viterbi_spec.h:25-35),
median of 10 wall-clock runs in ms (benchmark_helper.h:14,37-66).  One JSON line per cell.

Per cell:
  ms          median of 10 passes over the whole file, model resident in HBM (batch upload of the
              symbols, one launch, scores back to the host: svh_viterbi)
  ms_setup    non-spec only: the same plus svh_model_create inside every run, as the reference
              times run_Viterbi with its per-call model build (bench_Viterbi.h:53-56)
  prep_ms     spec only: spec_with (svh_spec_build), timed apart as bench_Viterbi_spec.h:69-71
  check       "digests": every sequence bit-exact against the committed oracle digests where they
              exist (tests/golden/scope_digests.json: every model x emit_3_3500_20, non-spec and
              level 2; score_digests.json: 2405 x emit_50 / covid-19, 100 x emit_3, 2405 x emit_50
              level 2; sweep2_digests.json: level 2 of every model x the other three files); otherwise the first sequence against the CPU oracle, "bit-exact", or for
              level 2 on models with n > 600 (the oracle's products would take minutes)
              "almost_equal-L0" (every sequence within HMM::almost_equal of the non-spec scores)

    python3 tools/bench_sweep.py [--models 100.chmm,2405.chmm] [--levels 0,1,2] [--out FILE]
"""
from __future__ import annotations

import argparse
import glob
import hashlib
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import spec_viterbi_amd as svh  # noqa: E402
from oracle import oracle  # noqa: E402  (the checker)
from tests.helpers import bit_equal  # noqa: E402

DATASETS = ["emit_3_3500_20.ess", "emit_3_7000_20.ess", "covid-19.ess", "emit_50_3500_20.ess"]
RUNS = 10


def digest_rows(model: str, dataset: str, level: int):
    """SHA-256 digests of the oracle's rows for this cell (level 0/1 share the non-spec rows), or None."""
    g = os.path.join(ROOT, "tests", "golden")
    with open(os.path.join(g, "scope_digests.json")) as f:
        scope = json.load(f)
    with open(os.path.join(g, "score_digests.json")) as f:
        sd = json.load(f)
    if dataset == scope["ess"] and model in scope["models"]:
        key = "scores_sha256" if level <= 1 else "spec2_sha256" if level == 2 else None
        if key:
            return [r[key] for r in scope["models"][model]]
    k = f"{model} x {dataset}" + ("" if level <= 1 else f" level {level}")
    if k in sd:
        return [r["scores_sha256"] for r in sd[k]]
    with open(os.path.join(g, "sweep2_digests.json")) as f:  # level 2 of the other files
        s2 = json.load(f)
    return s2.get(k)


def timed(fn, runs=RUNS):
    out = []
    for _ in range(runs):
        t0 = time.perf_counter()
        fn()
        out.append((time.perf_counter() - t0) * 1e3)
    return statistics.median(out)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--models", default="")
    p.add_argument("--datasets", default=",".join(DATASETS))
    p.add_argument("--levels", default="0,1,2")
    p.add_argument("--out", default="")
    a = p.parse_args()
    models = a.models.split(",") if a.models else sorted(
        (os.path.basename(f) for f in glob.glob(os.path.join(ROOT, "data", "chmm_files", "*.chmm"))),
        key=lambda s: int(s.split(".")[0]))
    levels = [int(x) for x in a.levels.split(",")]
    sink = open(a.out, "w") if a.out else None
    data = {d: svh.read_emit_seq(os.path.join(ROOT, "data", "ess_files", d)) for d in a.datasets.split(",")}
    for name in models:
        hmm = svh.read_HMM(os.path.join(ROOT, "data", "chmm_files", name))
        n = int(hmm.states_num)
        model = svh.DeviceModel(hmm)
        info = model.info()
        for lv in levels:
            prep_ms = None
            if lv >= 1:
                t0 = time.perf_counter()
                model.spec_build(lv)
                prep_ms = (time.perf_counter() - t0) * 1e3
            for dname, seqs in data.items():
                model.viterbi(seqs, level=lv)  # warm-up
                ms = timed(lambda: model.viterbi(seqs, level=lv))
                ms_setup = None
                if lv == 0:
                    def with_setup():
                        m = svh.DeviceModel(hmm)
                        m.viterbi(seqs)
                        m.close()
                    ms_setup = timed(with_setup)
                scores, _ = model.viterbi(seqs, level=lv)
                ref = digest_rows(name, dname, lv)
                if ref is not None:
                    ok = len(ref) == len(seqs) and all(
                        hashlib.sha256(np.ascontiguousarray(scores[q], np.float32).tobytes()).hexdigest() == ref[q]
                        for q in range(len(seqs)))
                    check = "digests" if ok else "MISMATCH"
                elif lv <= 1:
                    ok = bit_equal(scores[0], oracle.viterbi(hmm, seqs[0]))
                    check = "bit-exact" if ok else "MISMATCH"
                elif n <= 600:
                    ok = bit_equal(scores[0], oracle.viterbi_spec(hmm, lv, seqs[0]))
                    check = "bit-exact" if ok else "MISMATCH"
                else:
                    base, _ = model.viterbi(seqs, level=0)
                    fin = np.isfinite(base)
                    ok = bool(np.array_equal(fin, np.isfinite(scores)) and np.all(np.abs(scores[fin] - base[fin]) <= 1.0))
                    check = "almost_equal-L0" if ok else "MISMATCH"
                obs = sum(int(s.size) for s in seqs)
                rec = {"model": name, "states": n, "dataset": dname, "sequences": len(seqs), "observations": obs,
                       "level": lv, "ms": round(ms, 3), "ms_setup": None if ms_setup is None else round(ms_setup, 3),
                       "prep_ms": None if prep_ms is None else round(prep_ms, 3),
                       "M_state_updates_per_s": round(n * obs / ms / 1e3, 1),
                       "kernel": info["kernel"], "check": check}
                line = json.dumps(rec)
                print(line, flush=True)
                if sink:
                    sink.write(line + "\n")
                    sink.flush()
                if not ok:
                    raise SystemExit(f"bench_sweep: {name} x {dname} level {lv}: output check failed")
        model.close()


if __name__ == "__main__":
    main()
