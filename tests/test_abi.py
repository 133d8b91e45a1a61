"""The C-ABI library: loads on a CPU-only host and exports every entry point of include/mm360.h.
No compute call is made here (no GPU)."""
import ctypes
import os
import re

import numpy as np
import pytest

import mm360
from helpers import ROOT


def _header_functions():
    text = open(os.path.join(ROOT, "include", "mm360.h")).read()
    return sorted(set(re.findall(r"^(?:int|int64_t|void|const char\*|mm_epipole_list\*)\s+(mm_\w+)\(", text, re.M)))


def test_header_and_binding_agree():
    assert sorted(mm360.EXPORTED_SYMBOLS) == _header_functions()


def test_library_exports_every_symbol():
    lib = mm360.load_library()
    for name in _header_functions():
        assert hasattr(lib, name), name


def test_version():
    assert mm360.load_library().mm_get_version() == 300


def test_create_without_gpu_fails_loudly():
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("a GPU is present")
    except ImportError:
        pass
    with pytest.raises(mm360.MMError) as e:
        mm360.MMContext(mm360.seq_params(256, 128, [1]))
    assert e.value.code in (mm360.MM_ERR_NODEV, mm360.MM_ERR_HIP)


def test_struct_layouts_match_header():
    text = open(os.path.join(ROOT, "include", "mm360.h")).read()
    body = re.search(r"typedef struct mm_seq_params \{(.*?)\}", text, re.S).group(1)
    n_fields = sum(len(re.findall(r"\w+\s*(?:,|;)", l.split("/*")[0])) for l in body.splitlines() if ";" in l)
    assert ctypes.sizeof(mm360.SeqParams) == 4 * n_fields == 36
    assert mm360.BLOCK_DTYPE.itemsize == 40 and mm360.PU_DTYPE.itemsize == 64
    # mm_pic_job (mm_pred_device_multi): natural C alignment on LP64
    assert ctypes.sizeof(mm360.PicJob) == 64
    assert [getattr(mm360.PicJob, f).offset for f in ("cur_poc", "d_pus", "n", "dst_y", "dst_stride_y", "dst_cb",
                                                      "dst_cr", "dst_stride_c")] == [0, 8, 16, 24, 32, 40, 48, 56]


def test_product_has_no_oracle_dependency():
    """The product never imports, links or includes the oracle."""
    pkg = os.path.join(ROOT, "vvc-extension-mm_amd")
    for dp, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".h", ".hip", ".cpp", "Makefile")):
                txt = open(os.path.join(dp, f)).read()
                assert "oracle" not in txt.lower() or f == "__init__.py" and "oracle" not in txt, f


def test_cpp_shim_example_builds_and_fails_loudly_without_gpu():
    """The C++ host shim (host/mm360_vtm.hpp) compiles against the C-ABI; without a GPU the
    example exits through the shim's exception with MM_ERR_NODEV (no CPU fallback)."""
    import subprocess
    pkg = os.path.join(ROOT, "vvc-extension-mm_amd")
    subprocess.check_call(["make", "-s", "-C", pkg, "example"])
    exe = os.path.join(pkg, "lib", "example_decode")
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present: covered by tests/test_gpu.py::test_cpp_shim_example_on_gpu")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 2, r.stdout + r.stderr
    assert "mm360 error 6" in r.stdout


def test_build_provenance_record():
    """bench.py's `build` key: the library's and the sources' sha256 against __graft_entry__.build()'s record."""
    from mm360 import provenance
    assert provenance.source_sha256() == provenance.source_sha256()
    rel = [os.path.relpath(f, ROOT) for f in provenance.source_files()]
    assert "include/mm360.h" in rel and "vvc-extension-mm_amd/csrc/mm_kernels.hip" in rel
    if os.path.exists(mm360.LIB_PATH):
        p = provenance.provenance(mm360.LIB_PATH)
        assert len(p["lib_sha256"]) == 64 and len(p["src_sha256"]) == 64
        assert "built_by_build" in p or "build_info" in p
