#!/usr/bin/env python3
"""Time-parallel pass (svh_batch_run_time_parallel) on a ragged batch: time, segments re-run and
the largest relative score difference against the serial (bit-exact) pass, per (seg, probe)."""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import spec_viterbi_amd as svh  # noqa: E402


def main():
    model_name = os.environ.get("TP_MODEL", "2405.chmm")
    ess_name = os.environ.get("TP_ESS", "covid-19.ess")
    hmm = svh.read_HMM(os.path.join(ROOT, "data", "chmm_files", model_name))
    seqs = svh.read_emit_seq(os.path.join(ROOT, "data", "ess_files", ess_name))
    model = svh.DeviceModel(hmm)
    batch = model.batch(seqs)
    times = []
    for _ in range(7):
        batch.run()
        times.append(batch.elapsed_ms())
    ref, ref_best = batch.read()
    print(f"{model_name} x {ess_name}: serial {statistics.median(times):.4f} ms", flush=True)
    fin = np.isfinite(ref)
    for spec in sys.argv[1:] or ["1024,256", "512,128", "256,64"]:
        seg, probe = map(int, spec.split(","))
        times = []
        for _ in range(7):
            fb = batch.run_time_parallel(seg, probe)
            times.append(batch.elapsed_ms())
        s, b = batch.read()
        err = float(np.max(np.abs(s[fin] - ref[fin]) / np.maximum(1.0, np.abs(ref[fin]))))
        print(f"seg {seg:5d} probe {probe:4d}: {statistics.median(times):.4f} ms  re-run segments {fb}  "
              f"max rel diff {err:.2e}  best equal {bool(np.array_equal(b, ref_best))}  "
              f"inf pattern equal {bool(np.array_equal(np.isfinite(s), fin))}", flush=True)


if __name__ == "__main__":
    main()
