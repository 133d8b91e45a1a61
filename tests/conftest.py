import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "vvc-extension-mm_amd"), ROOT, os.path.join(ROOT, "tests", "native")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP library through the C-ABI)")


@pytest.fixture(scope="session", autouse=True)
def _native_builds():
    """Make sure the oracle and the CPU twin are built (cheap no-op when up to date)."""
    for d in ("oracle", os.path.join("tests", "native")):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, d)])
    subprocess.check_call(["make", "-s", "-j4", "-C", os.path.join(ROOT, "tests", "native"), "variants"])
    yield


GOLDEN = os.path.join(ROOT, "tests", "golden")
