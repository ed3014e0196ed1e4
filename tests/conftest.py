import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "eager-sgd_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

LIB = os.path.join(PKG, "esgd", "libesgd.so")
ORACLE = os.path.join(ROOT, "oracle", "libffref.so")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu)")
    config.addinivalue_line("markers", "slow: multi-process or large-size test")
    # Build on first use (here; the GPU box receives the prebuilt .so files).
    if not os.path.exists(ORACLE):
        subprocess.check_call(["make", "-C", ROOT, "oracle"])
    if not os.path.exists(LIB):
        subprocess.check_call(["make", "-C", ROOT, "-j8", "lib"])


@pytest.fixture(scope="session")
def golden_dir():
    return os.path.join(ROOT, "tests", "golden")
