"""The drop-in's per-call host glue (dcol_amd._fastpair, csrc/fastpair.c) on the CPU.

Engine.solve_pair calls dcol_prox_pair through this extension once both primitives are
known.  Here the library entry point is replaced by a ctypes callback of the same C
signature (include/dcol.h dcol_prox_pair), so the pose marshalling -- float64 arrays, lists,
(3, 1) arrays, strided views, integers, numpy scalars -- the argument order, the outputs and
the "not 3 numbers" refusal are checked without a GPU.
"""
import ctypes

import numpy as np
import pytest

from conftest import REPO  # noqa: F401  (puts the package on sys.path)

PROTO = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32,
                         ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double), ctypes.c_double,
                         ctypes.c_int32, ctypes.c_int32, ctypes.POINTER(ctypes.c_double),
                         ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                         ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32))


@pytest.fixture()
def fake():
    from dcol_amd import _fastpair   # built by __graft_entry__.build() (csrc/Makefile)
    seen = {}

    def impl(table, s1, s2, p1, p2, tol, max_iter, flags, alpha, contact, grad, iters, status):
        seen.update(table=table, s1=s1, s2=s2, pose=[p1[k] for k in range(6)] + [p2[k] for k in range(6)], tol=tol,
                    max_iter=max_iter, flags=flags)
        alpha[0] = 1.25
        if contact:
            for k in range(3):
                contact[k] = 10.0 + k
        if grad:
            for k in range(12):
                grad[k] = -1.0 - k
        iters[0] = 7
        status[0] = 0
        return seen.get("rc", 0)

    cb = PROTO(impl)
    addr = ctypes.cast(cb, ctypes.c_void_p).value
    return _fastpair, addr, seen, cb


def test_marshalling_and_outputs(fake):
    fp, addr, seen, _cb = fake
    from dcol_amd import _lib
    r1 = np.array([1.0, 2.0, 3.0])
    p1 = [0.1, 0.2, 0.3]                                   # lists (piano_mover.py:176)
    r2 = np.arange(6.0)[::2]                               # a strided view: item by item
    p2 = np.array([[4.0], [5.0], [6.0]])                   # (3, 1): contiguous, 3 values
    out = fp.solve(addr, 0x1234, 3, 5, r1, p1, r2, p2, 1e-6, 50, _lib.GRAD_FD, False)
    rc, alpha, contact, grad, iters, status = out
    assert rc == 0 and iters == 7 and status == 0
    assert isinstance(alpha, np.float64) and alpha == 1.25
    assert contact is None
    assert isinstance(grad, np.ndarray) and grad.dtype == np.float64 and grad.shape == (12,)
    np.testing.assert_array_equal(grad, -1.0 - np.arange(12))
    assert seen["table"] == 0x1234 and seen["s1"] == 3 and seen["s2"] == 5
    assert seen["pose"] == [1.0, 2.0, 3.0, 0.1, 0.2, 0.3, 0.0, 2.0, 4.0, 4.0, 5.0, 6.0]
    assert seen["tol"] == 1e-6 and seen["max_iter"] == 50 and seen["flags"] == _lib.GRAD_FD
    # proximity_mrp's form: contact, no gradient; ints and numpy scalars as coordinates
    rc, alpha, contact, grad, _, _ = fp.solve(addr, 1, 0, 1, [1, 2, 3], (np.float64(0.5), np.float32(0.25), 0),
                                              np.zeros(3), np.ones(3), 1e-5, 9, _lib.CONTACT, True)
    np.testing.assert_array_equal(contact, [10.0, 11.0, 12.0])
    assert grad is None
    assert seen["pose"][:6] == [1.0, 2.0, 3.0, 0.5, 0.25, 0.0]


def test_error_code_passed_through(fake):
    fp, addr, seen, _cb = fake
    seen["rc"] = -3
    rc, alpha, contact, grad, _, _ = fp.solve(addr, 1, 0, 1, np.zeros(3), np.zeros(3), np.zeros(3), np.zeros(3),
                                              1e-6, 50, 1, True)
    assert rc == -3 and contact is None and grad is None    # the caller raises with dcol_last_error


@pytest.mark.parametrize("bad", [np.zeros(4), [1.0, 2.0], "abc", None, np.zeros(3, dtype=np.complex128),
                                 [[1.0], [2.0], [3.0]]])
def test_not_three_numbers_refused(fake, bad):
    """anything but 3 numbers: None, and Engine.solve_pair takes its Python path (which
    reshapes nested lists or raises like the reference)"""
    fp, addr, seen, _cb = fake
    assert fp.solve(addr, 1, 0, 1, bad, np.zeros(3), np.zeros(3), np.zeros(3), 1e-6, 50, 0, False) is None
    assert "pose" not in seen
