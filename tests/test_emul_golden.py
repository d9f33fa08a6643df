"""x86 build of the device solver (tests/emul, LPP = 1) against the reference's golden
vectors -- checks the kernel's arithmetic without a GPU.  Skipped unless the emulator has
been built (`make -C tests/emul -j8`, ~3.5 min of hipcc host compilation, one object per
(N, NSOC) and row form)."""
import ctypes
import os

import numpy as np
import pytest

from conftest import REPO, alpha_close, golden_files, grad_close, load_golden

LIB = os.path.join(REPO, "tests", "emul", "libdcol_emul.so")
pytestmark = pytest.mark.skipif(not os.path.exists(LIB), reason="tests/emul not built")


def emul(d, tol, flags, max_iter=50):
    from dcol_amd import make_descs, spec_from_arrays
    lib = ctypes.CDLL(LIB)
    P = ctypes.c_void_p
    specs = [spec_from_arrays(d, k) for k in range(len(d["type"]))]
    descs, keep = make_descs(specs)
    B = len(d["s1"])
    s1 = np.ascontiguousarray(d["s1"], np.int32)
    s2 = np.ascontiguousarray(d["s2"], np.int32)
    p1 = np.ascontiguousarray(d["pose1"])
    p2 = np.ascontiguousarray(d["pose2"])
    al, ct, gr = np.empty(B), np.empty((B, 3)), np.empty((B, 12))
    it, st = np.empty(B, np.int32), np.empty(B, np.int32)
    rc = lib.dcol_emul_batch(descs, ctypes.c_int32(len(specs)), ctypes.c_int64(B), P(s1.ctypes.data),
                             P(s2.ctypes.data), P(p1.ctypes.data), P(p2.ctypes.data), ctypes.c_double(tol),
                             ctypes.c_int32(max_iter), ctypes.c_int32(flags), P(al.ctypes.data), P(ct.ctypes.data),
                             P(gr.ctypes.data), P(it.ctypes.data), P(st.ctypes.data))
    assert rc == 0
    return al, ct, gr, it, st


@pytest.mark.parametrize("orth_rows", ["partitioned", "dense"])
@pytest.mark.parametrize("soc_rows", ["structured", "dense"])
@pytest.mark.parametrize("flags", [1 | 4, 2 | 4], ids=["fd", "envelope"])
@pytest.mark.parametrize("path", [p for p in golden_files() if "tol0" not in p], ids=lambda p: p.split("/")[-1][:-4])
def test_emulated_kernel_matches_reference(path, flags, soc_rows, orth_rows, monkeypatch):
    """Both SOC row forms: structured blocks (Solver<..., BALL> for cone-free SOC pairs,
    Solver<..., CONE> for ball-free N = 4 pairs -- what the GPU plans run) and the dense rows
    (DCOL_NO_BALL, DCOL_NO_CONE); both orthant row forms: the row-partitioned N = 5 / 6
    buckets (Solver<..., OE>, what the GPU plans run) and the dense rows (DCOL_NO_PART)."""
    for var in ("DCOL_NO_BALL", "DCOL_NO_CONE"):
        if soc_rows == "dense":
            monkeypatch.setenv(var, "1")
        else:
            monkeypatch.delenv(var, raising=False)
    if orth_rows == "dense":
        monkeypatch.setenv("DCOL_NO_PART", "1")
    else:
        monkeypatch.delenv("DCOL_NO_PART", raising=False)
    d = load_golden(path)
    al, ct, gr, it, st = emul(d, float(d["tol"]), flags)
    np.testing.assert_array_equal(st, d["status"])
    ok = d["status"] == 0
    np.testing.assert_array_equal(it[ok], d["iters"][ok])
    assert np.all(alpha_close(al[ok], d["alpha"][ok]))
    if not np.all(np.isnan(d["grad"])):
        assert np.all(grad_close(gr[ok], d["grad"][ok]))
