#!/usr/bin/env python3
"""Split of the host-to-host time of one batched Viterbi call on 2405.chmm x emit_50_3500_20.

Times (median of N, ms): the one-shot call from a Python list of uint64 arrays (svh_viterbi_seqs,
no flattening), from packed uint8 symbols (svh_viterbi_u8, the device format), from packed uint64
(pack_sequences + svh_viterbi: the round-3 path), the Python packing alone, the kernel alone (HIP
events, batch resident), and the result read alone (D2H into pinned staging, sync, copy out).
Every result is checked against the committed digests.

    python3 tools/e2e_split.py [--reps 20]
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import spec_viterbi_amd as svh  # noqa: E402
from spec_viterbi_amd import _lib  # noqa: E402
from spec_viterbi_amd.hmm import pack_sequences  # noqa: E402
from spec_viterbi_amd.viterbi import _f32, _i64, _p, _u64  # noqa: E402
from tests.helpers import load_digests  # noqa: E402


def med(f, reps):
    f()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        f()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)) * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    hmm = svh.read_HMM(os.path.join(ROOT, "data", "chmm_files", "2405.chmm"))
    seqs = svh.read_emit_seq(os.path.join(ROOT, "data", "ess_files", "emit_50_3500_20.ess"))
    rows = load_digests()["2405.chmm x emit_50_3500_20.ess"]
    model = svh.DeviceModel(hmm, device=0)

    def ok(scores):
        return all(hashlib.sha256(np.ascontiguousarray(scores[q], np.float32).tobytes()).hexdigest()
                   == rows[q]["scores_sha256"] for q in range(len(rows)))

    offs, sym64 = pack_sequences(seqs)
    sym8 = sym64.astype(np.uint8)
    res = {}
    res["list_seqs_ms"] = med(lambda: model.viterbi(seqs), a.reps)
    res["packed_u8_ms"] = med(lambda: model.viterbi_packed(offs, sym8), a.reps)
    pout = (svh.pinned_empty((len(seqs), model.n), np.float32), svh.pinned_empty(len(seqs), np.int64))
    res["packed_u8_pinned_out_ms"] = med(lambda: model.viterbi_packed(offs, sym8, out=pout), a.reps)
    res["packed_u64_ms"] = med(lambda: model.viterbi_packed(offs, sym64), a.reps)

    def old_path():  # round 3: pack in Python, then svh_viterbi
        o, s = pack_sequences(seqs)
        sc = np.empty((len(seqs), model.n), np.float32)
        be = np.empty(len(seqs), np.int64)
        _lib.check(_lib.lib.svh_viterbi(model.handle, 0, len(seqs), _p(o, _u64), _p(s, _u64), _p(sc, _f32),
                                        _p(be, _i64), None))
        return sc
    res["pack_plus_u64_ms"] = med(old_path, a.reps)
    res["python_pack_ms"] = med(lambda: pack_sequences(seqs), a.reps)
    checks = {"list": ok(model.viterbi(seqs)[0]), "u8": ok(model.viterbi_packed(offs, sym8)[0]),
              "u8_pinned": ok(model.viterbi_packed(offs, sym8, out=pout)[0]),
              "u64": ok(model.viterbi_packed(offs, sym64)[0]), "old": ok(old_path())}

    batch = model.batch(seqs)
    ks = []
    for _ in range(a.reps + 1):
        batch.run()
        ks.append(batch.elapsed_ms())
    res["kernel_ms"] = float(np.median(ks[1:]))

    def read():
        batch.read()
    batch.run()
    batch.read()
    res["read_ms"] = med(read, a.reps)

    def run_sync():
        batch.run()
        batch.read()
    res["run_plus_read_ms"] = med(run_sync, a.reps)
    res["checks"] = checks
    res["overhead_list_ms"] = res["list_seqs_ms"] - res["kernel_ms"]
    res["overhead_u8_ms"] = res["packed_u8_ms"] - res["kernel_ms"]
    res["overhead_u8_pinned_out_ms"] = res["packed_u8_pinned_out_ms"] - res["kernel_ms"]
    print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in res.items()}), flush=True)
    batch.close()
    model.close()
    if not all(checks.values()):
        raise SystemExit("e2e_split: a result differs from the digests")


if __name__ == "__main__":
    main()
