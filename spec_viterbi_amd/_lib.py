"""ctypes binding of the C ABI in include/svh.h (libspec_viterbi_hip.so, built in-tree).

The product path has no fallback: if the HIP library is missing this module raises at import
time, loudly, instead of silently computing on the CPU.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_float, c_int, c_int32, c_int64, c_uint32, c_uint64, c_void_p

LIB_NAME = "libspec_viterbi_hip.so"
LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), LIB_NAME)
# A/B timing of alternative builds of the same engine (tools/ab_lib.sh): another in-tree build of
# this library, never a fallback (it must exist, or import fails as for the default).
if os.environ.get("SVH_LIB"):
    LIB_PATH = os.path.abspath(os.environ["SVH_LIB"])

SVH_OK = 0
SVH_E_INVALID = -1
SVH_E_RANGE = -2
SVH_E_NOMEM = -3
SVH_E_HIP = -4
SVH_E_UNSUPPORTED = -5
SVH_E_STATE = -6
SVH_E_IO = -7

SVH_KERNEL_AUTO = 0
SVH_KERNEL_FUSED = 1
SVH_KERNEL_GENERIC = 2
SVH_KERNEL_BAND = 3
SVH_KERNEL_CHAIN = 4
SVH_KERNEL_PIPE = 5
SVH_KERNEL_PIPE_WIDE = 6
SVH_KERNEL_SPEC2 = 7  # svh_batch_plan only: _spec level 2 on chip
SVH_KERNEL_SPEC2_PIPE = 8  # svh_batch_plan only: _spec level 2 on the pipelined latency plan
SVH_KERNEL_DIAG = 9  # the diagonal plan (diag.hip): scores-only passes, no inter-wave exchange
SVH_BATCH_PATHS = 1
SVH_BATCH_NO_TIMING = 2  # no start/stop events per run (svh_batch_elapsed_ms unavailable)
SVH_MODEL_SPEC_DENSE = 1


class SvhError(RuntimeError):
    """Non-zero status from the C ABI; `code` is the SVH_E_* value."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"svh error {code}: {msg}")
        self.code = code


class svh_model_opts(ctypes.Structure):
    _fields_ = [("device", c_int32), ("kernel", c_int32), ("max_threads", c_int32), ("flags", c_int32)]


class svh_model_info(ctypes.Structure):
    _fields_ = [
        ("kernel", c_int32), ("family", c_int32), ("threads", c_int32), ("slots", c_int32),
        ("light_terms", c_int32), ("heavy_rows", c_int32), ("heavy_uniform", c_int32), ("device", c_int32),
        ("n", c_uint64), ("S", c_uint64), ("nnz", c_uint64), ("lds_bytes", c_uint64),
        ("spec_level", c_uint64), ("spec_bytes", c_uint64), ("paths_kernel", c_int32), ("wide_threads", c_int32),
        ("wide_slots", c_int32), ("cu_count", c_uint32), ("pipe_slots", c_int32), ("pipe_waves", c_int32),
        ("pipe_groups", c_int32), ("pipe_max_nseq", c_uint32),
        ("pipew_slots", c_int32), ("pipew_waves", c_int32), ("pipew_blocks", c_int32), ("pipew_min_nseq", c_uint32),
        ("pipe_max_nseq_paths", c_uint32),
        ("diag_ranges", c_int32),
        ("diag_max_nseq", c_uint32),
    ]


P_u64 = POINTER(c_uint64)
P_f32 = POINTER(c_float)
P_i64 = POINTER(c_int64)
P_i32 = POINTER(c_int32)
P_u32 = POINTER(c_uint32)

# name -> (restype, argtypes); every function declared in include/svh.h.
SIGNATURES = {
    "svh_abi_version": (c_int, []),
    "svh_last_error": (c_char_p, []),
    "svh_device_count": (c_int, [P_i32]),
    "svh_hmm_read": (c_int, [c_char_p, POINTER(c_void_p)]),
    "svh_hmm_dims": (c_int, [c_void_p, P_u64, P_u64, P_u64, P_u64]),
    "svh_hmm_copy": (c_int, [c_void_p, P_u64, P_f32, P_f32, P_u64, P_u64, P_f32]),
    "svh_hmm_free": (None, [c_void_p]),
    "svh_ess_read": (c_int, [c_char_p, POINTER(c_void_p)]),
    "svh_ess_dims": (c_int, [c_void_p, P_u64, P_u64]),
    "svh_ess_copy": (c_int, [c_void_p, P_u64, P_u64]),
    "svh_ess_free": (None, [c_void_p]),
    "svh_model_create": (c_int, [c_uint64, c_uint64, c_uint64, P_u64, P_f32, P_f32, c_uint64, P_u64,
                                 P_u64, P_f32, POINTER(svh_model_opts), POINTER(c_void_p)]),
    "svh_model_destroy": (c_int, [c_void_p]),
    "svh_model_get_info": (c_int, [c_void_p, POINTER(svh_model_info)]),
    "svh_spec_build": (c_int, [c_void_p, c_uint32, c_void_p]),
    "svh_batch_create": (c_int, [c_void_p, c_uint64, P_u64, P_u64, c_uint32, POINTER(c_void_p)]),
    "svh_batch_run": (c_int, [c_void_p, c_uint32, c_void_p]),
    "svh_batch_read": (c_int, [c_void_p, c_void_p, P_f32, P_i64, P_i32]),
    "svh_host_alloc": (c_int, [ctypes.c_size_t, POINTER(c_void_p)]),
    "svh_host_free": (c_int, [c_void_p]),
    "svh_batch_device_results": (c_int, [c_void_p, POINTER(c_void_p), POINTER(c_void_p)]),
    "svh_batch_elapsed_ms": (c_int, [c_void_p, P_f32]),
    "svh_batch_step_floor_ms": (c_int, [c_void_p, c_void_p, c_uint32, P_f32]),
    "svh_batch_fallback_rows": (c_int, [c_void_p, P_u32]),
    "svh_batch_plan": (c_int, [c_void_p, c_uint32, POINTER(svh_model_info)]),
    "svh_batch_fallbacks": (c_int, [c_void_p, P_u64]),
    "svh_pipe_variant_built": (c_int, [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, POINTER(ctypes.c_int32)]),
    "svh_batch_debug_fault": (c_int, [c_void_p, c_void_p]),
    "svh_batch_destroy": (c_int, [c_void_p]),
    "svh_viterbi": (c_int, [c_void_p, c_uint32, c_uint64, P_u64, P_u64, P_f32, P_i64, P_i32]),
    "svh_viterbi_u8": (c_int, [c_void_p, c_uint32, c_uint64, P_u64, POINTER(ctypes.c_uint8), P_f32, P_i64, P_i32]),
    "svh_viterbi_seqs": (c_int, [c_void_p, c_uint32, c_uint64, P_u64, P_u64, P_f32, P_i64, P_i32]),
    "svh_batch_create_u8": (c_int, [c_void_p, c_uint64, P_u64, POINTER(ctypes.c_uint8), c_uint32, POINTER(c_void_p)]),
    "svh_batch_run_time_parallel": (c_int, [c_void_p, c_uint32, c_uint32, c_float, c_void_p, P_u64]),
    "svh_reader_open": (c_int, [c_char_p, c_int, POINTER(c_void_p)]),
    "svh_reader_next": (c_int, [c_void_p, c_uint64, c_uint64, P_u64, POINTER(P_u64),
                                POINTER(POINTER(ctypes.c_uint8))]),
    "svh_reader_close": (None, [c_void_p]),
    "svh_decode_file": (c_int, [c_void_p, c_char_p, c_int, c_uint32, c_uint32, c_uint64, c_uint64, c_void_p,
                                c_void_p, P_u64]),
}

SVH_FORMAT_AUTO, SVH_FORMAT_ESS, SVH_FORMAT_FASTA = 0, 1, 2
# int (*svh_result_fn)(void*, uint64 first, uint64 nseq, const uint64* offsets, const float* scores,
#                      const int64* best, const int32* paths)
RESULT_FN = ctypes.CFUNCTYPE(c_int, c_void_p, c_uint64, c_uint64, P_u64, P_f32, P_i64, P_i32)


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} not found: build the HIP extension first (python -c 'import __graft_entry__ as g; g.build()' "
            "or `make -j16`). There is no CPU fallback.")
    # One HIP runtime per process, shared with PyTorch: torch's bundled libamdhip64 and ours have
    # the same soname, so whichever loads first serves both.  Loading ours first and letting torch
    # initialise the GPU afterwards left our hipGetDevice reporting no device (seen on MI355X), so
    # torch, when present, loads first.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


lib = _load()


def check(rc: int) -> None:
    if rc != SVH_OK:
        msg = lib.svh_last_error()
        raise SvhError(rc, msg.decode() if msg else "")


def device_count() -> int:
    c = c_int32(0)
    check(lib.svh_device_count(ctypes.byref(c)))
    return int(c.value)


def pipe_variant_built(slots: int, waves: int, table_mode: int) -> bool:
    """svh_pipe_variant_built: is this latency-kernel variant in the loaded build?"""
    r = ctypes.c_int32()
    check(lib.svh_pipe_variant_built(slots, waves, table_mode, ctypes.byref(r)))
    return bool(r.value)
