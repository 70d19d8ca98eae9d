"""Streaming ingestion: the input side of the path for large batches.

Sequence files are read incrementally by the native reader (spec_viterbi_amd/csrc/stream.cpp,
C ABI svh_reader_* / svh_decode_file):
  * .ess   -- read_emit_seq semantics (reference Viterbi_impl/data_reader.cpp:93-134);
  * FASTA  -- ess_files/fasta_to_ess.py semantics (reference ess_files/fasta_to_ess.py:3-45):
              ACDEFGHIKLMNPQRSTVWY -> 0..19, X -> 0, '>' starts a sequence; an empty line or a
              residue outside the table is an error (the script's IndexError / KeyError).
`decode_file` runs the pipelined decoder: parsing on a host thread ahead of the GPU, chunk k's
kernels overlapping chunk k-1's result copies.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib

_FORMATS = {"auto": _lib.SVH_FORMAT_AUTO, "ess": _lib.SVH_FORMAT_ESS, "fasta": _lib.SVH_FORMAT_FASTA}


def _fmt(fmt) -> int:
    if isinstance(fmt, int):
        return fmt
    try:
        return _FORMATS[str(fmt).lower()]
    except KeyError:
        raise ValueError(f"format must be one of {sorted(_FORMATS)}") from None


class SeqReader:
    """Iterate over a sequence file in chunks of whole sequences: (offsets uint64 [nseq+1],
    symbols uint8) per chunk, at most max_seqs sequences / max_symbols symbols each."""

    def __init__(self, path, fmt="auto", max_seqs: int = 4096, max_symbols: int = 1 << 22):
        self.max_seqs = int(max_seqs)
        self.max_symbols = int(max_symbols)
        h = ctypes.c_void_p()
        _lib.check(_lib.lib.svh_reader_open(str(path).encode(), _fmt(fmt), ctypes.byref(h)))
        self._h = h

    def __iter__(self):
        return self

    def __next__(self):
        if not self._h:
            raise StopIteration
        n = ctypes.c_uint64()
        offs = ctypes.POINTER(ctypes.c_uint64)()
        syms = ctypes.POINTER(ctypes.c_uint8)()
        _lib.check(_lib.lib.svh_reader_next(self._h, self.max_seqs, self.max_symbols, ctypes.byref(n),
                                            ctypes.byref(offs), ctypes.byref(syms)))
        if n.value == 0:
            self.close()
            raise StopIteration
        o = np.ctypeslib.as_array(offs, shape=(n.value + 1,)).copy()
        s = np.ctypeslib.as_array(syms, shape=(int(o[-1]),)).copy() if o[-1] else np.zeros(0, np.uint8)
        return o, s

    def close(self):
        if getattr(self, "_h", None):
            _lib.lib.svh_reader_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def read_sequences(path, fmt="auto") -> list[np.ndarray]:
    """A whole file as a list of uint64 symbol arrays (the shape read_emit_seq returns)."""
    out = []
    for offs, syms in SeqReader(path, fmt):
        out.extend(syms[offs[q]:offs[q + 1]].astype(np.uint64) for q in range(offs.size - 1))
    return out


def decode_file(model, path, fmt="auto", level: int = 0, paths: bool = False, max_seqs: int = 4096,
                max_symbols: int = 1 << 22):
    """Pipelined decode of a whole file on `model` (a DeviceModel): returns scores [N, n],
    best states [N] and (with paths) the decoded paths, in file order."""
    scores, best, pth = [], [], []

    def on_chunk(_user, first, nseq, offsets, sc, be, pa):
        try:
            o = np.ctypeslib.as_array(offsets, shape=(nseq + 1,))
            scores.append(np.ctypeslib.as_array(sc, shape=(nseq, model.n)).copy())
            best.append(np.ctypeslib.as_array(be, shape=(nseq,)).copy())
            if paths:
                p = np.ctypeslib.as_array(pa, shape=(int(o[-1]),)) if o[-1] else np.zeros(0, np.int32)
                pth.extend(p[o[q]:o[q + 1]].copy() for q in range(nseq))
            return 0
        except Exception:  # never unwind through the C frame
            return 1

    cb = _lib.RESULT_FN(on_chunk)
    total = ctypes.c_uint64()
    _lib.check(_lib.lib.svh_decode_file(model.handle, str(path).encode(), _fmt(fmt), int(level),
                                        _lib.SVH_BATCH_PATHS if paths else 0, int(max_seqs), int(max_symbols),
                                        ctypes.cast(cb, ctypes.c_void_p), None, ctypes.byref(total)))
    s = np.concatenate(scores) if scores else np.zeros((0, model.n), np.float32)
    b = np.concatenate(best) if best else np.zeros(0, np.int64)
    if len(s) != total.value:
        raise RuntimeError("decode_file: result hand-off stopped early")
    return (s, b, pth) if paths else (s, b)
