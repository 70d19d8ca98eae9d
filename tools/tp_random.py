#!/usr/bin/env python3
"""Time-parallel pass on random ergodic models (tests/helpers.random_hmm): segments re-run and the
largest relative score difference against the serial pass."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import spec_viterbi_amd as svh  # noqa: E402
from tests.helpers import random_chain_hmm, random_hmm, random_seqs  # noqa: E402

for name, hmm in [("random_hmm(300,deg4)", random_hmm(300, out_degree=4, seed=3)),
                  ("random_hmm(1000,deg8)", random_hmm(1000, out_degree=8, seed=4)),
                  ("random_chain_hmm(300)", random_chain_hmm(300, seed=1))]:
    seqs = random_seqs(hmm.emit_num, [8000, 6000, 4000, 100], seed=5)
    model = svh.DeviceModel(hmm)
    batch = model.batch(seqs)
    batch.run()
    t_ser = batch.elapsed_ms()
    ref, rb = batch.read()
    fin = np.isfinite(ref)
    for seg, probe in [(1024, 256), (512, 128), (512, 32)]:
        fb = batch.run_time_parallel(seg, probe)
        t = batch.elapsed_ms()
        s, b = batch.read()
        err = float(np.max(np.abs(s[fin] - ref[fin]) / np.maximum(1.0, np.abs(ref[fin]))))
        nseg = sum(max(1, len(x) // seg) if len(x) > 2 * seg else 1 for x in seqs) - len(seqs)
        print(f"{name:24s} kernel {model.info()['kernel']} serial {t_ser:.3f} ms | seg {seg} probe {probe}: "
              f"{t:.3f} ms re-run {fb}/{nseg} max rel diff {err:.1e} best equal {np.array_equal(b, rb)}", flush=True)
