"""CPU: the host readers under AddressSanitizer + UBSan (tests/cpp/test_readers_asan.cpp)."""
import os
import subprocess

import pytest

from tests.conftest import DATA, ROOT

BIN = os.path.join(ROOT, "tests", "cpp", "test_readers_asan")


def test_readers_under_asan(tmp_path):
    if not os.path.exists(BIN):
        pytest.skip("tests/cpp/test_readers_asan not built (make tests)")
    fasta = os.path.join(ROOT, "tests", "golden", "covid-19.fasta")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([BIN, DATA, fasta, str(tmp_path)], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ok" in r.stdout


HOST_BIN = os.path.join(ROOT, "tests", "cpp", "test_host_asan")


def test_host_code_under_asan(tmp_path):
    """The rest of the host code under AddressSanitizer + UBSan (tests/cpp/test_host_asan.cpp): the
    host CSR and every plan builder over the 24 .chmm and 240 generated models plus malformed ones,
    and the file decoder's chunk hand-off (chunker.cpp) with a consumer thread over the .ess files
    and the FASTA fixture, including a file that fails mid-way.  Leak checking stays on."""
    if not os.path.exists(HOST_BIN):
        pytest.skip("tests/cpp/test_host_asan not built (make tests)")
    fasta = os.path.join(ROOT, "tests", "golden", "covid-19.fasta")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([HOST_BIN, DATA, fasta, str(tmp_path)], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failures" in r.stdout and "24 models" in r.stdout, r.stdout
