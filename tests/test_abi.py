"""CPU: the C-ABI library loads and exports every symbol include/svh.h declares."""
import ctypes
import os
import re

import spec_viterbi_amd._lib as L
from tests.conftest import ROOT


def declared_symbols():
    text = open(os.path.join(ROOT, "include", "svh.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|void|const char\*)\s+(svh_\w+)\s*\(", text, re.M)))


def test_header_and_binding_agree():
    decl = declared_symbols()
    assert len(decl) >= 20
    assert sorted(L.SIGNATURES) == decl


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(L.LIB_PATH)
    for name in declared_symbols():
        assert hasattr(lib, name), name


def test_abi_version_and_error_channel():
    assert L.lib.svh_abi_version() == 4
    h = ctypes.c_void_p()
    rc = L.lib.svh_hmm_read(b"/nonexistent.chmm", ctypes.byref(h))
    assert rc == L.SVH_E_IO
    assert b"cannot open" in L.lib.svh_last_error()


def test_cpp_classes_exported():
    # HIP_impl / HIP_spec_impl (include/HIP_impl.h, HIP_spec_impl.h) live in the same library
    import subprocess
    out = subprocess.run(["nm", "-DC", L.LIB_PATH], capture_output=True, text=True).stdout
    for sym in ["HIP_impl::run_Viterbi", "HIP_spec_impl::spec_with", "HIP_spec_impl::run_Viterbi_spec",
                "read_HMM(", "read_emit_seq("]:
        assert sym in out, sym


def test_model_create_rejects_nan_and_minus_inf_scores():
    """-log2 p is finite or +inf; NaN / -inf scores are refused before any device call
    (kernels are built with -fno-honor-nans; see runtime.cpp build_host_model)."""
    import numpy as np

    u64 = ctypes.POINTER(ctypes.c_uint64)
    f32 = ctypes.POINTER(ctypes.c_float)
    n, S = 2, 1
    sc = np.array([0], np.uint64)
    src = np.array([0, 1], np.uint64)
    dst = np.array([1, 0], np.uint64)
    for bad in (float("nan"), float("-inf")):
        for where in ("start", "emis", "trans"):
            sv = np.array([1.0 if where != "start" else bad], np.float32)
            em = np.array([0.5, 0.5 if where != "emis" else bad], np.float32)
            pr = np.array([1.0, 2.0 if where != "trans" else bad], np.float32)
            opts = L.svh_model_opts(-1, 0, 0, 0)
            h = ctypes.c_void_p()
            rc = L.lib.svh_model_create(n, S, 1, sc.ctypes.data_as(u64), sv.ctypes.data_as(f32),
                                        em.ctypes.data_as(f32), 2, src.ctypes.data_as(u64), dst.ctypes.data_as(u64),
                                        pr.ctypes.data_as(f32), ctypes.byref(opts), ctypes.byref(h))
            assert rc == L.SVH_E_INVALID, (bad, where, rc)
            assert b"NaN or -inf" in L.lib.svh_last_error()


def test_hmm_fingerprint_tracks_content():
    import numpy as np

    import spec_viterbi_amd as svh
    from spec_viterbi_amd.viterbi import hmm_fingerprint
    from tests.conftest import chmm

    a = svh.read_HMM(chmm("100.chmm"))
    b = svh.read_HMM(chmm("100.chmm"))
    c = svh.read_HMM(chmm("200.chmm"))
    assert hmm_fingerprint(a) == hmm_fingerprint(b) != hmm_fingerprint(c)
    b.trans_probs = b.trans_probs + np.float32(0.5)
    assert hmm_fingerprint(a) != hmm_fingerprint(b)
