"""HMM value model and .chmm/.ess readers.

Mirrors the reference's `class HMM` (reference: Viterbi_impl/HMM.h:7-60) and its readers
`read_HMM` / `read_emit_seq` (Viterbi_impl/data_reader.h:8,11).  Parsing is done by the engine's
native C++ reader (spec_viterbi_amd/csrc/data_reader.cpp via the C ABI) so fp32 parsing and the
-log2 mapping are bit-identical to the reference's iostream + std::log2(float) path.
"""
from __future__ import annotations

import ctypes
import math
from dataclasses import dataclass, field

import numpy as np

from . import _lib

ZERO_PROB = math.inf  # HMM::zero_prob (HMM.h:41)


def to_modified_prob(p: float) -> float:
    """-log2(p) in fp32 for p > 0, +inf otherwise (HMM.h:51-57)."""
    p32 = np.float32(p)
    if not p32 > 0:
        return ZERO_PROB
    return float(np.float32(-np.log2(p32)))


def almost_equal(x: float, y: float) -> bool:
    """The reference tolerance: both +inf or |x - y| <= 1.0 (HMM.h:43-49)."""
    if x == ZERO_PROB and y == ZERO_PROB:
        return True
    return abs(x - y) <= 1.0


@dataclass
class HMM:
    """Field names follow the reference class; arrays are numpy (indices uint64, probs float32)."""
    states_num: int
    emit_num: int
    trans_num: int
    trans_rows: np.ndarray          # source state of each transition
    trans_cols: np.ndarray          # destination state
    trans_probs: np.ndarray         # -log2 p
    emissions: np.ndarray           # [emit_num][states_num]
    start_probabilities_cols: np.ndarray
    start_probabilities: np.ndarray
    non_zero_start_probs: int = field(default=0)

    def __post_init__(self):
        self.trans_rows = np.ascontiguousarray(self.trans_rows, dtype=np.uint64)
        self.trans_cols = np.ascontiguousarray(self.trans_cols, dtype=np.uint64)
        self.trans_probs = np.ascontiguousarray(self.trans_probs, dtype=np.float32)
        self.emissions = np.ascontiguousarray(self.emissions, dtype=np.float32).reshape(
            self.emit_num, self.states_num)
        self.start_probabilities_cols = np.ascontiguousarray(self.start_probabilities_cols, dtype=np.uint64)
        self.start_probabilities = np.ascontiguousarray(self.start_probabilities, dtype=np.float32)
        self.non_zero_start_probs = int(self.start_probabilities.size)


def _ptr(a: np.ndarray, ctype):
    return a.ctypes.data_as(ctypes.POINTER(ctype))


def read_HMM(path: str) -> HMM:
    """Parse a .chmm file with the native reader (data_reader.cpp:17-79 semantics)."""
    h = ctypes.c_void_p()
    _lib.check(_lib.lib.svh_hmm_read(str(path).encode(), ctypes.byref(h)))
    try:
        n, S, ns, nt = (ctypes.c_uint64() for _ in range(4))
        _lib.check(_lib.lib.svh_hmm_dims(h, ctypes.byref(n), ctypes.byref(S), ctypes.byref(ns), ctypes.byref(nt)))
        n, S, ns, nt = n.value, S.value, ns.value, nt.value
        sc = np.zeros(ns, np.uint64)
        sv = np.zeros(ns, np.float32)
        em = np.zeros(S * n, np.float32)
        src = np.zeros(nt, np.uint64)
        dst = np.zeros(nt, np.uint64)
        pr = np.zeros(nt, np.float32)
        _lib.check(_lib.lib.svh_hmm_copy(h, _ptr(sc, ctypes.c_uint64), _ptr(sv, ctypes.c_float),
                                         _ptr(em, ctypes.c_float), _ptr(src, ctypes.c_uint64),
                                         _ptr(dst, ctypes.c_uint64), _ptr(pr, ctypes.c_float)))
    finally:
        _lib.lib.svh_hmm_free(h)
    return HMM(states_num=n, emit_num=S, trans_num=nt, trans_rows=src, trans_cols=dst, trans_probs=pr,
               emissions=em.reshape(S, n), start_probabilities_cols=sc, start_probabilities=sv)


def read_emit_seq(path: str) -> list[np.ndarray]:
    """Parse an .ess file (data_reader.cpp:93-134 semantics); one uint64 array per sequence."""
    h = ctypes.c_void_p()
    _lib.check(_lib.lib.svh_ess_read(str(path).encode(), ctypes.byref(h)))
    try:
        nseq, total = ctypes.c_uint64(), ctypes.c_uint64()
        _lib.check(_lib.lib.svh_ess_dims(h, ctypes.byref(nseq), ctypes.byref(total)))
        offsets = np.zeros(nseq.value + 1, np.uint64)
        symbols = np.zeros(total.value, np.uint64)
        _lib.check(_lib.lib.svh_ess_copy(h, _ptr(offsets, ctypes.c_uint64), _ptr(symbols, ctypes.c_uint64)))
    finally:
        _lib.lib.svh_ess_free(h)
    return [symbols[offsets[q]:offsets[q + 1]].copy() for q in range(nseq.value)]


def pack_sequences(seqs) -> tuple[np.ndarray, np.ndarray]:
    """Sequences -> (offsets[nseq+1], symbols) as contiguous uint64 arrays."""
    seqs = [np.ascontiguousarray(s, dtype=np.uint64) for s in seqs]
    offsets = np.zeros(len(seqs) + 1, np.uint64)
    if seqs:
        offsets[1:] = np.cumsum([s.size for s in seqs], dtype=np.uint64)
    symbols = np.concatenate(seqs) if seqs else np.zeros(0, np.uint64)
    return offsets, np.ascontiguousarray(symbols, dtype=np.uint64)
