"""Bit-exact numerics (csrc/mm_numerics.h) against this container's glibc 2.35 libm and the
Eigen 3.3.7 SSE packet kernels executed natively.

The full exhaustive run (every float, ~6 min on 8 cores) is recorded in
tests/golden/numerics_exhaustive_r01.txt; here a 1/61-stride sample of every function runs."""
import os
import subprocess

import pytest

from helpers import GOLDEN, ROOT


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    # one binary per test process (pytest -n workers must not overwrite each other's executable)
    check = str(tmp_path_factory.mktemp("numerics") / "mm360_check_numerics")
    src = os.path.join(ROOT, "tools", "check_numerics.cpp")
    inc = os.path.join(ROOT, "vvc-extension-mm_amd", "csrc")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-mfma", "-msse4.1", "-ffp-contract=off", "-fopenmp",
                           "-I", inc, src, "-o", check, "-lm"])
    return check


@pytest.mark.parametrize("fn", ["sinf", "cosf", "atanf", "acosf", "asinf", "tanf", "roundf", "dsin", "dcos",
                                "psin", "pcos", "psqrt", "atan2f"])
def test_function_sample_exact(checker, fn):
    out = subprocess.run([checker, "quick", fn], capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "ALL EXACT" in out.stdout


def test_exhaustive_log_committed():
    log = open(os.path.join(GOLDEN, "numerics_exhaustive_r01.txt")).read()
    assert "NUMERICS: ALL EXACT" in log
    for fn in ["sinf", "cosf", "atanf", "acosf", "asinf", "tanf", "roundf", "psin", "pcos", "psqrt"]:
        assert fn in log
    assert "mismatches 1" not in log and "mismatches 2" not in log
