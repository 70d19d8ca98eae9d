"""Reference-interface backends on the HIP engine.

`Viterbi_impl` / `Viterbi_spec_impl` mirror the reference's abstract classes
(Viterbi_impl/Viterbi_impl.h:6-11, Viterbi_spec_impl.h:6-24); `HIP_impl` / `HIP_spec_impl` are
the MI355X backends (same names as the C++ classes in include/HIP_impl.h, HIP_spec_impl.h).
`DeviceModel` / `DeviceBatch` expose the batched, HBM-resident API underneath (include/svh.h).
"""
from __future__ import annotations

import abc
import ctypes
import hashlib

import numpy as np

from . import _lib
from .hmm import HMM, pack_sequences

_u64 = ctypes.POINTER(ctypes.c_uint64)
_f32 = ctypes.POINTER(ctypes.c_float)
_i64 = ctypes.POINTER(ctypes.c_int64)
_i32 = ctypes.POINTER(ctypes.c_int32)
_u32 = ctypes.POINTER(ctypes.c_uint32)


def _p(a, t):
    return a.ctypes.data_as(t)


def pinned_empty(shape, dtype=np.float32) -> np.ndarray:
    """An uninitialised array in page-locked host memory (svh_host_alloc): result buffers the DMA
    engine writes directly (DeviceModel.viterbi_packed(out=...), DeviceBatch.read(out=...)), with
    no staging copy.  The memory is freed when the array (and every view of it) is gone."""
    import weakref

    dtype = np.dtype(dtype)
    n = int(np.prod(shape)) * dtype.itemsize
    ptr = ctypes.c_void_p()
    _lib.check(_lib.lib.svh_host_alloc(max(n, 1), ctypes.byref(ptr)))
    buf = (ctypes.c_uint8 * max(n, 1)).from_address(ptr.value)
    arr = np.frombuffer(buf, np.uint8, count=n).view(dtype).reshape(shape)
    weakref.finalize(buf, _lib.lib.svh_host_free, ptr.value)
    return arr


def _result_arrays(out, nseq: int, n: int):
    """(scores float32 [nseq, n], best int64 [nseq]): the caller's `out` pair, checked, or new arrays."""
    if out is None:
        return np.empty((nseq, n), np.float32), np.empty(nseq, np.int64)
    scores, best = out
    if (scores.shape != (nseq, n) or scores.dtype != np.float32 or not scores.flags.c_contiguous
            or best.shape != (nseq,) or best.dtype != np.int64 or not best.flags.c_contiguous):
        raise ValueError("out: (float32 [nseq, n], int64 [nseq]) C-contiguous arrays expected")
    return scores, best


class DeviceModel:
    """An HMM resident in HBM on one device (svh_model_create)."""

    def __init__(self, hmm: HMM, device: int = -1, kernel: int = _lib.SVH_KERNEL_AUTO, max_threads: int = 0,
                 flags: int = 0):
        self.n = int(hmm.states_num)
        self.S = int(hmm.emit_num)
        opts = _lib.svh_model_opts(device, kernel, max_threads, flags)
        h = ctypes.c_void_p()
        sc = np.ascontiguousarray(hmm.start_probabilities_cols, np.uint64)
        sv = np.ascontiguousarray(hmm.start_probabilities, np.float32)
        em = np.ascontiguousarray(hmm.emissions, np.float32)
        src = np.ascontiguousarray(hmm.trans_rows, np.uint64)
        dst = np.ascontiguousarray(hmm.trans_cols, np.uint64)
        pr = np.ascontiguousarray(hmm.trans_probs, np.float32)
        _lib.check(_lib.lib.svh_model_create(self.n, self.S, sc.size, _p(sc, _u64), _p(sv, _f32), _p(em, _f32),
                                             pr.size, _p(src, _u64), _p(dst, _u64), _p(pr, _f32),
                                             ctypes.byref(opts), ctypes.byref(h)))
        self._h = h

    @property
    def handle(self):
        return self._h

    def info(self) -> dict:
        i = _lib.svh_model_info()
        _lib.check(_lib.lib.svh_model_get_info(self._h, ctypes.byref(i)))
        return {name: getattr(i, name) for name, _ in i._fields_}

    def spec_build(self, level: int, stream: int | None = None) -> None:
        _lib.check(_lib.lib.svh_spec_build(self._h, int(level), ctypes.c_void_p(stream or 0)))

    def batch(self, seqs, paths: bool = False, timing: bool = True) -> "DeviceBatch":
        return DeviceBatch(self, seqs, paths, timing)

    def viterbi(self, seqs, level: int = 0, paths: bool = False):
        """One-shot: scores [nseq, n] (+ best state [nseq], + paths list if requested).
        uint64 sequences go to svh_viterbi_seqs as they are (no flattening here: the C side narrows
        each one straight into its pinned upload); anything else is packed first."""
        seqs = [s if isinstance(s, np.ndarray) and s.dtype == np.uint64 and s.flags.c_contiguous
                else np.ascontiguousarray(s, np.uint64) for s in seqs]
        nseq = len(seqs)
        lens = np.fromiter((s.size for s in seqs), np.uint64, nseq)
        ptrs = np.fromiter((s.ctypes.data for s in seqs), np.uint64, nseq)
        scores = np.empty((nseq, self.n), np.float32)
        best = np.empty(nseq, np.int64)
        pth = np.empty(int(lens.sum()), np.int32) if paths else None
        _lib.check(_lib.lib.svh_viterbi_seqs(self._h, int(level), nseq, _p(ptrs, _u64), _p(lens, _u64),
                                             _p(scores, _f32), _p(best, _i64), _p(pth, _i32) if paths else None))
        if paths:
            offsets = np.zeros(nseq + 1, np.int64)
            np.cumsum(lens, out=offsets[1:])
            return scores, best, [pth[offsets[q]:offsets[q + 1]] for q in range(nseq)]
        return scores, best

    def viterbi_packed(self, offsets, symbols, level: int = 0, paths: bool = False, out=None):
        """One-shot over packed sequences: offsets [nseq+1] and uint8 symbols (the device format,
        svh_viterbi_u8; e.g. what svh_reader_next returns) or uint64 symbols (svh_viterbi).
        `out` = (scores [nseq, n] float32, best [nseq] int64) to fill instead of new arrays;
        arrays from pinned_empty take the scores straight from the DMA engine."""
        offsets = np.ascontiguousarray(offsets, np.uint64)
        symbols = np.asarray(symbols)
        # the C ABI takes no symbol count: check here that every sequence lies inside `symbols`
        # (a short array or a bad offsets vector would otherwise be a native out-of-bounds read)
        if offsets.ndim != 1 or offsets.size < 1:
            raise ValueError("offsets: a 1-D array of nseq + 1 entries expected")
        if symbols.ndim != 1:
            raise ValueError("symbols: a 1-D array expected")
        if np.any(offsets[1:] < offsets[:-1]) or int(offsets[-1]) > symbols.size:
            raise ValueError("offsets must be non-decreasing with offsets[-1] <= symbols.size")
        nseq = offsets.size - 1
        scores, best = _result_arrays(out, nseq, self.n)
        pth = np.empty(int(offsets[-1] - offsets[0]) if nseq else 0, np.int32) if paths else None
        if symbols.dtype == np.uint8:
            symbols = np.ascontiguousarray(symbols)
            fn, sp = _lib.lib.svh_viterbi_u8, _p(symbols, ctypes.POINTER(ctypes.c_uint8))
        else:
            symbols = np.ascontiguousarray(symbols, np.uint64)
            fn, sp = _lib.lib.svh_viterbi, _p(symbols, _u64)
        _lib.check(fn(self._h, int(level), nseq, _p(offsets, _u64), sp, _p(scores, _f32), _p(best, _i64),
                      _p(pth, _i32) if paths else None))
        if paths:
            base = int(offsets[0])
            return scores, best, [pth[int(offsets[q]) - base:int(offsets[q + 1]) - base] for q in range(nseq)]
        return scores, best

    def close(self):
        if getattr(self, "_h", None):
            _lib.lib.svh_model_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class DeviceBatch:
    """Sequences resident in HBM; run() enqueues one pass on a HIP stream (svh_batch_*)."""

    def __init__(self, model: DeviceModel, seqs, paths: bool = False, timing: bool = True):
        """timing=False: run() records no start/stop events on the stream (SVH_BATCH_NO_TIMING;
        elapsed_ms() then raises) -- for callers that time the stream themselves."""
        self.model = model
        self.offsets, symbols = pack_sequences(seqs)
        self.nseq = self.offsets.size - 1
        self.paths = paths
        self.total = int(self.offsets[-1])
        h = ctypes.c_void_p()
        _lib.check(_lib.lib.svh_batch_create(model.handle, self.nseq, _p(self.offsets, _u64), _p(symbols, _u64),
                                             (_lib.SVH_BATCH_PATHS if paths else 0) |
                                             (0 if timing else _lib.SVH_BATCH_NO_TIMING), ctypes.byref(h)))
        self._h = h

    def run(self, level: int = 0, stream: int | None = None) -> None:
        _lib.check(_lib.lib.svh_batch_run(self._h, int(level), ctypes.c_void_p(stream or 0)))

    def run_time_parallel(self, seg_len: int = 1024, probe_len: int = 256, rel_tol: float = 1e-6,
                          stream: int | None = None) -> int:
        """Opt-in time-parallel scores (svh_batch_run_time_parallel): long sequences are cut into
        segments that run concurrently; scores match the serial pass up to rounding (measured up
        to 1.4e-5 relative on 2405 x covid-19, DESIGN.md 6b -- not bit-exact, unlike run()).
        `rel_tol` is the convergence check's tolerance (when a segment's probe counts as
        converged), not a bound on the output error; rel_tol < 0 re-runs every segment and is
        bit-exact.  Returns the number of segments re-run exactly.  On MSV-shaped models that the
        pipelined plan runs, the serial run() is faster (2405 x covid-19: 0.66 vs 0.90 ms); the
        pass pays on models the pipelined plans do not take."""
        fb = ctypes.c_uint64()
        _lib.check(_lib.lib.svh_batch_run_time_parallel(self._h, int(seg_len), int(probe_len), float(rel_tol),
                                                         ctypes.c_void_p(stream or 0), ctypes.byref(fb)))
        return int(fb.value)

    def read(self, stream: int | None = None, want_paths: bool = False, out=None):
        """Scores [nseq, n] and best states [nseq] (+ paths) of the last run.  `out` = (scores,
        best) to fill instead of new arrays (same checks as DeviceModel.viterbi_packed); arrays from
        pinned_empty take the D2H copy directly."""
        scores, best = _result_arrays(out, self.nseq, self.model.n)
        pth = np.empty(self.total, np.int32) if want_paths else None
        _lib.check(_lib.lib.svh_batch_read(self._h, ctypes.c_void_p(stream or 0), _p(scores, _f32), _p(best, _i64),
                                           _p(pth, _i32) if want_paths else None))
        if want_paths:
            return scores, best, [pth[self.offsets[q]:self.offsets[q + 1]] for q in range(self.nseq)]
        return scores, best

    def device_results(self) -> tuple[int, int]:
        s, b = ctypes.c_void_p(), ctypes.c_void_p()
        _lib.check(_lib.lib.svh_batch_device_results(self._h, ctypes.byref(s), ctypes.byref(b)))
        return int(s.value or 0), int(b.value or 0)

    def plan(self, level: int = 0) -> dict:
        """The plan run(level) launches for this batch (svh_batch_plan): model info fields with
        kernel / threads / slots of the narrow or wide chain plan this batch selects."""
        i = _lib.svh_model_info()
        _lib.check(_lib.lib.svh_batch_plan(self._h, int(level), ctypes.byref(i)))
        return {name: getattr(i, name) for name, _ in i._fields_}

    def fallbacks(self) -> int:
        """Rows of the last run that the pipelined kernel re-ran on the serial chain kernel
        (svh_batch_fallbacks; 0 if the last run did not use the pipelined kernel)."""
        r = ctypes.c_uint64()
        _lib.check(_lib.lib.svh_batch_fallbacks(self._h, ctypes.byref(r)))
        return int(r.value)

    def fallback_rows(self) -> np.ndarray:
        """Per row (svh_batch_fallback_rows): bit 0 the step pass re-ran it exactly, bit 1 the
        level-2 pipelined pass handed it to the on-chip chunk kernel."""
        f = np.zeros(self.nseq, np.uint32)
        _lib.check(_lib.lib.svh_batch_fallback_rows(self._h, _p(f, _u32)))
        return f

    def debug_fault(self, stream: int | None = None) -> None:
        """Diagnostics (svh_batch_debug_fault): mark the last run as if a bounded wait had given
        up; this batch's next read() raises, other batches of the model are unaffected."""
        _lib.check(_lib.lib.svh_batch_debug_fault(self._h, ctypes.c_void_p(stream or 0)))

    def step_floor_ms(self, reps: int = 10, stream: int | None = None) -> float:
        """The latency plan's pass with every boundary exchange removed (svh_batch_step_floor_ms):
        the step's own per-observation time, the roofline the exchange is measured against.  Leaves
        the batch's results untouched."""
        ms = ctypes.c_float()
        _lib.check(_lib.lib.svh_batch_step_floor_ms(self._h, ctypes.c_void_p(stream or 0), int(reps), ctypes.byref(ms)))
        return float(ms.value)

    def elapsed_ms(self) -> float:
        ms = ctypes.c_float()
        _lib.check(_lib.lib.svh_batch_elapsed_ms(self._h, ctypes.byref(ms)))
        return float(ms.value)

    def close(self):
        if getattr(self, "_h", None):
            _lib.lib.svh_batch_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Viterbi_impl(abc.ABC):
    """Reference: Viterbi_impl/Viterbi_impl.h:6-11."""

    @abc.abstractmethod
    def run_Viterbi(self, hmm: HMM, seq) -> np.ndarray:
        ...


class Viterbi_spec_impl(abc.ABC):
    """Reference: Viterbi_impl/Viterbi_spec_impl.h:6-24."""

    def __init__(self, level: int):
        self.level = int(level)

    @abc.abstractmethod
    def spec_with(self, hmm: HMM) -> None:
        ...

    @abc.abstractmethod
    def run_Viterbi_spec(self, seq) -> np.ndarray:
        ...

    def get_level(self) -> int:
        return self.level


def hmm_fingerprint(hmm: HMM) -> bytes:
    """Content digest of an HMM (every field the device model is built from): equal digests <=>
    the same device model.  The C++ HIP_impl compares a host copy field by field instead
    (HIP_impl.cpp ModelKey); both rebuild the model for a different or modified HMM."""
    h = hashlib.blake2b(digest_size=16)
    h.update(np.array([hmm.states_num, hmm.emit_num], np.uint64).tobytes())
    for a in (hmm.trans_rows, hmm.trans_cols, hmm.trans_probs, hmm.emissions, hmm.start_probabilities_cols,
              hmm.start_probabilities):
        a = np.ascontiguousarray(a)
        h.update(np.array([a.size], np.uint64).tobytes())
        h.update(a.tobytes())
    return h.digest()


class HIP_impl(Viterbi_impl):
    """MI355X backend of Viterbi_impl.  The device model is cached by the HMM's content
    fingerprint (not its identity: a freed HMM's id can be reused, and an HMM can be changed in
    place), so every call runs the HMM it was given, as GraphBLAS_impl::run_Viterbi does
    (GraphBLAS_impl.cpp:9-54 builds the model from its argument on every call)."""

    def __init__(self, device: int = -1, **model_opts):
        self.device = device
        self.model_opts = model_opts
        self._cache: tuple[bytes, DeviceModel] | None = None

    def _model(self, hmm: HMM) -> DeviceModel:
        key = hmm_fingerprint(hmm)
        if self._cache is None or self._cache[0] != key:
            if self._cache is not None:
                self._cache[1].close()
            self._cache = (key, DeviceModel(hmm, self.device, **self.model_opts))
        return self._cache[1]

    def run_Viterbi(self, hmm: HMM, seq) -> np.ndarray:
        return self._model(hmm).viterbi([seq])[0][0]

    def run_Viterbi_batch(self, hmm: HMM, seqs) -> np.ndarray:
        return self._model(hmm).viterbi(seqs)[0]

    def decode_path(self, hmm: HMM, seq) -> np.ndarray:
        return self._model(hmm).viterbi([seq], paths=True)[2][0]


class HIP_spec_impl(Viterbi_spec_impl):
    """MI355X backend of Viterbi_spec_impl (level >= 2: products precomputed in HBM)."""

    def __init__(self, level: int, device: int = -1, **model_opts):
        super().__init__(level)
        self.device = device
        self.model_opts = model_opts
        self._model: DeviceModel | None = None

    def spec_with(self, hmm: HMM) -> None:
        self._model = DeviceModel(hmm, self.device, **self.model_opts)
        self._model.spec_build(self.level)

    def run_Viterbi_spec(self, seq) -> np.ndarray:
        return self.run_Viterbi_spec_batch([seq])[0]

    def run_Viterbi_spec_batch(self, seqs) -> np.ndarray:
        if self._model is None:
            raise RuntimeError("run_Viterbi_spec before spec_with")
        return self._model.viterbi(seqs, level=self.level)[0]
