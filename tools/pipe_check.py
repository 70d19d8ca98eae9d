"""Pipelined kernel vs the serial chain kernel on the GPU: identical scores / best states, and
kernel times (HIP events) of both, on reference workloads and on a random MSV model whose feeder
row does take its light term (so the speculation fails and the fallback runs).

    python tools/pipe_check.py [--reps 20]
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from spec_viterbi_amd import _lib  # noqa: E402
from spec_viterbi_amd.hmm import HMM, read_emit_seq, read_HMM  # noqa: E402
from spec_viterbi_amd.viterbi import DeviceModel  # noqa: E402

ROOT = os.path.join(os.path.dirname(__file__), "..", "data")


def msv_model(L: int, S: int, rng, cheap_loop: bool) -> HMM:
    """N, M_1..M_L, C with N <-> M_j (J loop), M_j -> M_j+1, M_j -> C, self loops on N and C."""
    n = L + 2
    rows, cols, probs = [], [], []

    def add(a, b, p):
        rows.append(a); cols.append(b); probs.append(p)

    add(0, 0, 0.5 if not cheap_loop else 0.01)
    add(n - 1, n - 1, 0.9)
    for j in range(1, L + 1):
        add(0, j, 1.0 / L)
        if j < L:
            add(j, j + 1, 0.8)
        add(j, n - 1, 0.05)
        add(j, 0, 0.05 if not cheap_loop else 0.9)
    em = (-np.log2(rng.dirichlet(np.ones(S) * 0.3, size=n).T)).astype(np.float32)  # [S][n], -log2 p
    h = HMM(states_num=n, emit_num=S, trans_num=len(rows),
            trans_rows=np.array(rows, np.uint64), trans_cols=np.array(cols, np.uint64),
            trans_probs=(-np.log2(np.array(probs, np.float64))).astype(np.float32), emissions=em,
            start_probabilities_cols=np.array([0], np.uint64), start_probabilities=np.array([0.0], np.float32),
            non_zero_start_probs=1)
    return h


def same(a, b):
    return np.array_equal(np.where(a == 0, 0, a), np.where(b == 0, 0, b))


def run(h, seqs, kernel, reps):
    m = DeviceModel(h, kernel=kernel)
    bt = m.batch(seqs)
    plan = bt.plan()
    bt.run()
    s, b = bt.read()
    ts = []
    for _ in range(reps):
        bt.run()
        ts.append(bt.elapsed_ms())
    s2, b2 = bt.read()
    assert same(s, s2) and np.array_equal(b, b2), "rerun differs"
    return s, b, float(np.median(ts)), plan


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    cases = [("2405", "emit_50_3500_20"), ("2405", "covid-19"), ("100", "emit_3_3500_20"),
             ("1509", "emit_3_7000_20"), ("2405", "emit_3_3500_20")]
    ok = True
    for mname, ename in cases:
        h = read_HMM(os.path.join(ROOT, "chmm_files", f"{mname}.chmm"))
        seqs = read_emit_seq(os.path.join(ROOT, "ess_files", f"{ename}.ess"))
        sc, bc, tc, _ = run(h, seqs, _lib.SVH_KERNEL_CHAIN, a.reps)
        sp, bp, tp, plan = run(h, seqs, _lib.SVH_KERNEL_PIPE, a.reps)
        eq = same(sc, sp) and np.array_equal(bc, bp)
        ok &= eq
        print(f"{mname} x {ename}: nseq {len(seqs)} chain {tc:.3f} ms pipe {tp:.3f} ms "
              f"(x{tc / tp:.2f}) equal={eq} plan kernel={plan['kernel']} slots={plan['slots']} "
              f"waves={plan['pipe_waves']} groups={plan['pipe_groups']}", flush=True)
    rng = np.random.default_rng(5)
    for cheap in (False, True):
        h = msv_model(300, 20, rng, cheap)
        seqs = [rng.integers(0, 20, size=int(x)) for x in rng.integers(1, 3000, size=12)]
        sc, bc, tc, _ = run(h, seqs, _lib.SVH_KERNEL_CHAIN, 3)
        sp, bp, tp, _ = run(h, seqs, _lib.SVH_KERNEL_PIPE, 3)
        eq = same(sc, sp) and np.array_equal(bc, bp)
        ok &= eq
        print(f"random MSV L=300 cheap_loop={cheap}: chain {tc:.3f} ms pipe {tp:.3f} ms equal={eq}", flush=True)
    print("ALL EQUAL" if ok else "MISMATCH")
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
