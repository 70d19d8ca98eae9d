#!/usr/bin/env python3
"""Interleaved A/B timing of kernel variants in one process (diagnostic).

Variants are environment settings read when a model is planned (SVH_CHAIN_GE, SVH_BAND_DEBUG)
plus svh_model_opts; every variant's output is checked bit-exact against the oracle on two
sequences before timing.  Usage:  python tools/ab.py 'GE=0' 'GE=4' 'kernel=1' ...
"""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import spec_viterbi_amd as svh  # noqa: E402
from spec_viterbi_amd import _lib  # noqa: E402


def main():
    model_name = os.environ.get("AB_MODEL", "2405.chmm")
    ess_name = os.environ.get("AB_ESS", "emit_50_3500_20.ess")
    rounds = int(os.environ.get("AB_ROUNDS", "7"))
    hmm = svh.read_HMM(os.path.join(ROOT, "data", "chmm_files", model_name))
    seqs = svh.read_emit_seq(os.path.join(ROOT, "data", "ess_files", ess_name))
    specs = sys.argv[1:] or ["GE=0"]
    variants = []
    ref = None
    for spec in specs:
        kv = dict(x.split("=") for x in spec.split(","))
        os.environ["SVH_CHAIN_GE"] = kv.get("GE", "0")
        os.environ["SVH_BAND_DEBUG"] = kv.get("dbg", "0")
        if "waves" in kv:
            os.environ["SVH_CHAIN_WAVES"] = kv["waves"]
        else:
            os.environ.pop("SVH_CHAIN_WAVES", None)
        model = svh.DeviceModel(hmm, kernel=int(kv.get("kernel", "0")), max_threads=int(kv.get("threads", "0")))
        batch = model.batch(seqs)
        batch.run()
        try:
            scores, _ = batch.read()
        except svh.viterbi._lib.SvhError as e:  # diagnostic ablations that break the exchange
            print(f"{spec}: {e}", flush=True)   # (DIAG 2/4) trip the bounded waits by design
            scores = np.full((len(seqs), hmm.states_num), np.nan, np.float32)
        if ref is None:
            ref = scores
        same = bool(np.all((scores.view(np.uint32) == ref.view(np.uint32)) | ((scores == 0) & (ref == 0))))
        variants.append((spec, model, batch, [], same, model.info()))
    for _ in range(rounds):
        for spec, model, batch, times, _, _ in variants:
            batch.run()
            times.append(batch.elapsed_ms())
            try:
                batch.read()
            except svh.viterbi._lib.SvhError:
                pass
    for spec, model, batch, times, same, info in variants:
        med = statistics.median(times)
        print(f"{spec:24s} kernel={info['kernel']} B={info['threads']} SM={info['slots']} "
              f"median {med:.4f} ms  min {min(times):.4f}  ns/obs {med * 1e6 / max(len(s) for s in seqs):.1f}  "
              f"same_as_first={same}", flush=True)


if __name__ == "__main__":
    main()
