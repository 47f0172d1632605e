"""C ABI checks that need no GPU: libsgc_amd.so loads and exports exactly the
entry points include/sgc_amd.h declares, with the ctypes signatures the
Python layer binds."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "sgc_amd.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(sgc_\w+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    from sgc_amd import build
    build.build(verbose=False)
    from sgc_amd import _lib
    return _lib.load()


def test_header_declares_core_api():
    names = declared_functions()
    for must in ("sgc_coo_to_csr", "sgc_spmm_csr_f32", "sgc_propagate_f32", "sgc_linear_f32",
                 "sgc_plan_build", "sgc_last_error", "sgc_abi_version"):
        assert must in names


def test_library_exports_every_declared_symbol(lib):
    from sgc_amd import _lib
    out = subprocess.check_output(["nm", "-D", "--defined-only", _lib.LIB_PATH], text=True)
    exported = {line.split()[-1] for line in out.splitlines() if line.strip()}
    missing = [n for n in declared_functions() if n not in exported]
    assert not missing, missing
    # every declared function is bound by the Python layer and vice versa
    assert sorted(_lib.SIGNATURES) == declared_functions()
    for name in declared_functions():
        assert getattr(lib, name) is not None


def test_host_only_entry_points(lib):
    assert lib.sgc_abi_version() == 1
    assert isinstance(lib.sgc_last_error(), bytes)
    assert lib.sgc_plan_capacity(1000) >= 2 * 1000 + 1
    assert lib.sgc_plan_capacity(-5) >= 1


def test_library_is_gfx950_code_object(lib):
    from sgc_amd import _lib
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data


def test_spmm_ex_accepts_every_declared_flag():
    """Every SGC_SPMM_* bit the header declares passes the flag check (the
    call then stops at its null pointers, before touching a device)."""
    import re
    from sgc_amd import _lib
    hdr = open(os.path.join(ROOT, "include", "sgc_amd.h")).read()
    bits = [int(v) for v in re.findall(r"SGC_SPMM_\w+ = (\d+)", hdr)]
    assert 128 in bits
    lib = _lib.load()
    for b in bits:
        rc = lib.sgc_spmm_csr_f32_ex(None, None, None, 0, 0, None, 1, None, 1, 1, None, 0, 0, 0,
                                     b, None)
        assert rc != 0 and b"unknown flags" not in lib.sgc_last_error(), b
