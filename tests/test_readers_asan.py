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
