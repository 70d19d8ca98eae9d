"""Shared helpers: golden loading, exact float comparison, synthetic models."""
from __future__ import annotations

import json
import os
import struct

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def load_golden(name):
    with open(os.path.join(GOLDEN, f"{name}.json")) as f:
        return json.load(f)


def load_digests():
    """tests/golden/score_digests.json: per-row SHA-256 of the oracle's float32 scores (+ paths)."""
    with open(os.path.join(GOLDEN, "score_digests.json")) as f:
        return json.load(f)


def from_hex(bits):
    return np.array([struct.unpack("<f", bytes.fromhex(b))[0] for b in bits], np.float32)


def bit_equal(a, b) -> bool:
    """Bit-exact fp32 equality, except that -0.0 == +0.0 (min of equal zeros may pick either)."""
    a = np.asarray(a, np.float32).ravel()
    b = np.asarray(b, np.float32).ravel()
    if a.shape != b.shape:
        return False
    ua, ub = a.view(np.uint32), b.view(np.uint32)
    same = ua == ub
    zeros = (a == 0) & (b == 0)
    return bool(np.all(same | zeros))


def first_mismatch(a, b):
    a = np.asarray(a, np.float32).ravel()
    b = np.asarray(b, np.float32).ravel()
    bad = np.nonzero(~((a.view(np.uint32) == b.view(np.uint32)) | ((a == 0) & (b == 0))))[0]
    if bad.size == 0:
        return None
    i = int(bad[0])
    return i, float(a[i]), float(b[i]), int(bad.size)


def random_hmm(n, S=20, out_degree=3, nstart=2, seed=0, dense_rows=(), self_loops=False, zero_emis=0.0):
    """chmm_gen.py-shaped random model (reference chmm_files/chmm_gen.py:1-62), seeded.

    dense_rows: states that every other state also transitions into (heavy rows).
    """
    from spec_viterbi_amd import HMM

    rng = np.random.default_rng(seed)
    nstart = min(nstart, n)

    def probs(k):
        w = rng.integers(1, 100, size=k).astype(np.float64)
        return (w / w.sum()).astype(np.float32)

    src, dst, pr = [], [], []
    for s in range(n):
        targets = rng.choice(n, size=min(out_degree, n), replace=False)
        for d, p in zip(targets, probs(targets.size)):
            src.append(s)
            dst.append(int(d))
            pr.append(p)
        if self_loops:
            src.append(s)
            dst.append(s)
            pr.append(np.float32(0.5))
    for d in dense_rows:
        for s in range(n):
            src.append(s)
            dst.append(d)
            pr.append(np.float32(0.01))
    em = np.stack([probs(S) for _ in range(n)]).T.copy()  # [S][n]
    if zero_emis > 0:
        em[rng.random(em.shape) < zero_emis] = 0.0

    def mod(p):
        p = np.asarray(p, np.float32)
        with np.errstate(divide="ignore"):
            return np.where(p > 0, -np.log2(p), np.inf).astype(np.float32)

    return HMM(states_num=n, emit_num=S, trans_num=len(pr), trans_rows=np.array(src, np.uint64),
               trans_cols=np.array(dst, np.uint64), trans_probs=mod(pr), emissions=mod(em),
               start_probabilities_cols=np.arange(nstart, dtype=np.uint64),
               start_probabilities=mod(probs(nstart)))


def random_seqs(S, lengths, seed=0):
    rng = np.random.default_rng(seed)
    return [rng.integers(0, S, size=int(L)).astype(np.uint64) for L in lengths]


def random_chain_hmm(L, S=20, seed=0, self_n=True, self_c=True, feed_c=False, c_from_m=True, n_from_m=True,
                     zero_emis=0.0, gap=None, start=(0,), ties=False, inf_edges=0.0, **_):
    """MSV-shaped random model (the shape chmm_files/silent_hmm_to_chmm.py writes): N=0, M_1..M_L,
    C=L+1.  N -> M_j, M_j -> M_{j+1}, M_j -> N and M_j -> C with one shared weight each, N and C
    self loops.  Variants: feed_c adds C -> M_j (light rows fed by two heavy rows); c_from_m /
    n_from_m drop the uniform M -> heavy terms; gap drops M_gap -> M_gap+1 (chain break); ties draws
    every probability from {1/2, 1/4, 1/8} (integer scores: exact ties everywhere); inf_edges sets
    that fraction of the light rows' terms to probability 0 (the term exists, weight +inf)."""
    from spec_viterbi_amd import HMM

    rng = np.random.default_rng(seed)
    n = L + 2
    C = L + 1
    src, dst, pr = [], [], []

    def add(a, b, p, shared=False):
        if ties and not shared:
            p = float(rng.choice([0.5, 0.25, 0.125]))
        if inf_edges > 0 and b not in (0, C) and rng.random() < inf_edges:
            p = 0.0
        src.append(a)
        dst.append(b)
        pr.append(np.float32(p))

    w_n, w_c = rng.uniform(0.01, 0.2), rng.uniform(0.01, 0.2)
    if ties:
        w_n, w_c = float(rng.choice([0.5, 0.25, 0.125])), float(rng.choice([0.5, 0.25, 0.125]))
    for j in range(1, L + 1):
        add(0, j, rng.uniform(0.001, 0.05))
        if feed_c:
            add(C, j, rng.uniform(0.001, 0.05))
        if j < L and j != gap:
            add(j, j + 1, rng.uniform(0.3, 0.9))
        if n_from_m:
            add(j, 0, w_n, shared=True)
        if c_from_m:
            add(j, C, w_c, shared=True)
    if self_n:
        add(0, 0, rng.uniform(0.5, 0.99))
    if self_c:
        add(C, C, rng.uniform(0.5, 0.99))
    em = rng.uniform(0.001, 1.0, size=(S, n)).astype(np.float32)
    if ties:
        em = rng.choice(np.array([0.5, 0.25, 0.125], np.float32), size=(S, n))
    if zero_emis > 0:
        em[rng.random(em.shape) < zero_emis] = 0.0

    def mod(p):
        p = np.asarray(p, np.float32)
        with np.errstate(divide="ignore"):
            return np.where(p > 0, -np.log2(p), np.inf).astype(np.float32)

    st = np.array(start, np.uint64)
    return HMM(states_num=n, emit_num=S, trans_num=len(pr), trans_rows=np.array(src, np.uint64),
               trans_cols=np.array(dst, np.uint64), trans_probs=mod(pr), emissions=mod(em),
               start_probabilities_cols=st, start_probabilities=mod(rng.uniform(0.1, 1.0, size=st.size)))
