import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

DATA = os.path.join(ROOT, "data")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C ABI)")


@pytest.fixture(scope="session")
def data_dir():
    return DATA


def chmm(name):
    return os.path.join(DATA, "chmm_files", name)


def ess(name):
    return os.path.join(DATA, "ess_files", name)
