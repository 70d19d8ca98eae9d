"""ctypes wrapper of the CPU oracle (oracle/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, as the checker / CPU baseline.  The product (spec_viterbi_amd/) never imports
it.  The algorithm restated, with reference file:line citations, is in viterbi_oracle.h/.c.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

_u64 = ctypes.POINTER(ctypes.c_uint64)
_f32 = ctypes.POINTER(ctypes.c_float)
_i32 = ctypes.POINTER(ctypes.c_int32)


class OraHMM(ctypes.Structure):
    _fields_ = [("n", ctypes.c_uint64), ("S", ctypes.c_uint64), ("nstart", ctypes.c_uint64),
                ("start_cols", _u64), ("start_vals", _f32), ("emis", _f32), ("ntrans", ctypes.c_uint64),
                ("src", _u64), ("dst", _u64), ("prob", _f32)]


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} missing: run `make oracle`")
    lib = ctypes.CDLL(LIB_PATH)
    P = ctypes.POINTER(OraHMM)
    lib.ora_viterbi.argtypes = [P, _u64, ctypes.c_uint64, _f32, _i32]
    lib.ora_traceback.argtypes = [ctypes.c_uint64, ctypes.c_uint64, _f32, _i32, _i32]
    lib.ora_argmin.argtypes = [ctypes.c_uint64, _f32]
    lib.ora_argmin.restype = ctypes.c_int64
    lib.ora_viterbi_spec.argtypes = [P, ctypes.c_uint32, _u64, ctypes.c_uint64, _f32]
    lib.ora_spec_products.argtypes = [P, ctypes.c_uint32, _f32]
    lib.ora_viterbi_spec_batch.argtypes = [P, ctypes.c_uint32, ctypes.c_uint64, _u64, _u64, _f32]
    lib.ora_viterbi_batch.argtypes = [P, ctypes.c_uint64, _u64, _u64, _f32, ctypes.c_int,
                                      ctypes.POINTER(ctypes.c_int)]
    return lib


lib = _load()


class _Model:
    """Keeps the numpy arrays alive while the C struct points at them."""

    def __init__(self, hmm):
        self.sc = np.ascontiguousarray(hmm.start_probabilities_cols, np.uint64)
        self.sv = np.ascontiguousarray(hmm.start_probabilities, np.float32)
        self.em = np.ascontiguousarray(hmm.emissions, np.float32).reshape(-1)
        self.src = np.ascontiguousarray(hmm.trans_rows, np.uint64)
        self.dst = np.ascontiguousarray(hmm.trans_cols, np.uint64)
        self.pr = np.ascontiguousarray(hmm.trans_probs, np.float32)
        self.n = int(hmm.states_num)
        self.S = int(hmm.emit_num)
        self.s = OraHMM(self.n, self.S, self.sc.size, self.sc.ctypes.data_as(_u64), self.sv.ctypes.data_as(_f32),
                        self.em.ctypes.data_as(_f32), self.pr.size, self.src.ctypes.data_as(_u64),
                        self.dst.ctypes.data_as(_u64), self.pr.ctypes.data_as(_f32))


def _rc(rc):
    if rc != 0:
        raise RuntimeError(f"oracle error {rc}")


def viterbi(hmm, seq, backpointers: bool = False):
    """GraphBLAS_impl::run_Viterbi restated: final scores [n] (+ bp [(len-1), n] int32)."""
    m = _Model(hmm)
    seq = np.ascontiguousarray(seq, np.uint64)
    out = np.empty(m.n, np.float32)
    bp = np.empty((max(seq.size - 1, 0), m.n), np.int32) if backpointers else None
    _rc(lib.ora_viterbi(ctypes.byref(m.s), seq.ctypes.data_as(_u64), seq.size, out.ctypes.data_as(_f32),
                        bp.ctypes.data_as(_i32) if backpointers else None))
    return (out, bp) if backpointers else out


def decode(hmm, seq):
    """(final scores, best final state, decoded path) with lowest-index tie-breaking."""
    scores, bp = viterbi(hmm, seq, backpointers=True)
    path = np.empty(len(seq), np.int32)
    _rc(lib.ora_traceback(scores.size, len(seq), scores.ctypes.data_as(_f32), bp.ctypes.data_as(_i32),
                          path.ctypes.data_as(_i32)))
    return scores, int(lib.ora_argmin(scores.size, scores.ctypes.data_as(_f32))), path


def viterbi_spec(hmm, level: int, seq):
    """GraphBLAS_spec_impl(level): spec_with + run_Viterbi_spec restated."""
    m = _Model(hmm)
    seq = np.ascontiguousarray(seq, np.uint64)
    out = np.empty(m.n, np.float32)
    _rc(lib.ora_viterbi_spec(ctypes.byref(m.s), int(level), seq.ctypes.data_as(_u64), seq.size,
                             out.ctypes.data_as(_f32)))
    return out


def viterbi_spec_batch(hmm, level: int, seqs):
    """viterbi_spec over many sequences with the products built once: scores [nseq, n]."""
    m = _Model(hmm)
    seqs = [np.ascontiguousarray(s, np.uint64) for s in seqs]
    offsets = np.zeros(len(seqs) + 1, np.uint64)
    offsets[1:] = np.cumsum([s.size for s in seqs])
    symbols = np.ascontiguousarray(np.concatenate(seqs), np.uint64)
    out = np.empty((len(seqs), m.n), np.float32)
    _rc(lib.ora_viterbi_spec_batch(ctypes.byref(m.s), int(level), len(seqs), offsets.ctypes.data_as(_u64),
                                   symbols.ctypes.data_as(_u64), out.ctypes.data_as(_f32)))
    return out


def spec_products(hmm, level: int):
    """Dense level-L products [S^L, n, n] (keys base-S, first symbol most significant)."""
    m = _Model(hmm)
    out = np.empty((m.S ** level, m.n, m.n), np.float32)
    _rc(lib.ora_spec_products(ctypes.byref(m.s), int(level), out.ctypes.data_as(_f32)))
    return out


def viterbi_batch(hmm, seqs, nthreads: int = 0):
    """Many sequences (OpenMP over sequences); returns (scores [nseq, n], threads used)."""
    m = _Model(hmm)
    seqs = [np.ascontiguousarray(s, np.uint64) for s in seqs]
    offsets = np.zeros(len(seqs) + 1, np.uint64)
    offsets[1:] = np.cumsum([s.size for s in seqs])
    symbols = np.ascontiguousarray(np.concatenate(seqs), np.uint64)
    out = np.empty((len(seqs), m.n), np.float32)
    used = ctypes.c_int(0)
    _rc(lib.ora_viterbi_batch(ctypes.byref(m.s), len(seqs), offsets.ctypes.data_as(_u64),
                              symbols.ctypes.data_as(_u64), out.ctypes.data_as(_f32), int(nthreads),
                              ctypes.byref(used)))
    return out, used.value
