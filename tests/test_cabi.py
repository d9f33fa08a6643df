"""C-ABI surface (no GPU needed): the library loads, exports every function declared in
include/dcol.h, and the ctypes signatures in dcol_amd._lib cover exactly that set."""
import os
import re
import subprocess

import pytest

from conftest import PKG, REPO

HEADER = os.path.join(REPO, "include", "dcol.h")


def declared_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(dcol_[a-z_0-9]+)\s*\(", txt)))


def test_header_declares_entry_points():
    fns = declared_functions()
    for f in ("dcol_table_create", "dcol_plan_create", "dcol_plan_run", "dcol_prox_batch_host"):
        assert f in fns


def test_library_exports_every_declared_symbol():
    from dcol_amd import _lib
    lib = _lib.load()
    for f in declared_functions():
        assert hasattr(lib, f), f
    assert set(_lib.SIGNATURES) == set(declared_functions())
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (dcol_\w+)", out))
    assert set(declared_functions()) <= exported


def test_host_only_entry_points():
    """Pure-host calls work without a device."""
    from dcol_amd import _lib
    lib = _lib.load()
    assert lib.dcol_abi_version() == _lib.ABI_VERSION
    assert _lib.status_string(_lib.MAXITER) == "Maximum number of iterations reached, PDIP failed"
    assert _lib.status_string(_lib.UNSUPPORTED) == "Failed to combine problem matrices."


def test_missing_library_fails_loudly(tmp_path):
    from dcol_amd import _lib
    with pytest.raises(_lib.DcolLibraryError):
        _lib.load(str(tmp_path / "nope.so"))


def test_stale_library_fails_with_version_error(tmp_path):
    """A library of an older ABI (here: a stand-in exporting only dcol_abi_version() = 3,
    none of the later entry points) is refused by its version, before any signature is
    bound -- a DcolLibraryError naming both versions, not an AttributeError."""
    from dcol_amd import _lib
    src = tmp_path / "stale.c"
    src.write_text("int dcol_abi_version(void) { return 3; }\n")
    so = tmp_path / "libstale.so"
    subprocess.run(["gcc", "-shared", "-fPIC", "-o", str(so), str(src)], check=True)
    with pytest.raises(_lib.DcolLibraryError, match=f"ABI version 3 != {_lib.ABI_VERSION}"):
        _lib.load(str(so))


def test_package_layout():
    for sub in ("proximity/proximity.py", "proximity/proximity_gradient.py", "primitives/misc_primitive_constructor.py",
                "dcol_amd/_lib.py", "csrc/dcol_device.hpp", "csrc/dcol_capi.cpp"):
        assert os.path.exists(os.path.join(PKG, sub)), sub


def test_header_constants_match_binding():
    """flag / size constants of include/dcol.h that dcol_amd._lib restates"""
    from dcol_amd import _lib
    txt = open(HEADER).read()

    def val(name):
        m = re.search(rf"\b{name}\s*=\s*(\d+)", txt) or re.search(rf"#define\s+{name}\s+(\d+)", txt)
        assert m, name
        return int(m.group(1))
    assert val("DCOL_NO_GATHER") == _lib.NO_GATHER
    assert val("DCOL_GRAD_IMPLICIT") == _lib.GRAD_IMPLICIT
    assert val("DCOL_CASE4") == _lib.CASE4
    assert val("DCOL_PAIR_PLANS_MAX") == _lib.PAIR_PLANS_MAX
    assert val("DCOL_ABI_VERSION") == _lib.ABI_VERSION
    assert val("DCOL_REC") == 14
