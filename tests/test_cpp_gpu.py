"""GPU: the C++ drop-in classes (HIP_impl / HIP_spec_impl) through the reference-style tests."""
import os
import subprocess

import pytest

from tests.conftest import DATA, ROOT

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["test_HIP_impl", "test_HIP_spec_impl", "test_semantic_equality"])
def test_cpp(name):
    exe = os.path.join(ROOT, "tests", "cpp", name)
    assert os.path.exists(exe), f"{exe} not built (make tests)"
    r = subprocess.run([exe, DATA], capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
