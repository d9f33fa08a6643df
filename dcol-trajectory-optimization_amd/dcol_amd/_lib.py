"""ctypes binding of the C-ABI in include/dcol.h (lib/libdcol.so, built in-tree).

The library is the product: there is no Python or CPU fallback.  If it cannot be loaded,
every entry point raises :class:`DcolLibraryError` (loudly, with the reason).
"""
from __future__ import annotations

import atexit
import ctypes
import os
from ctypes import POINTER, c_char_p, c_double, c_int, c_int32, c_int64, c_void_p

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("DCOL_LIB", os.path.join(PKG_ROOT, "lib", "libdcol.so"))

# enum dcol_shape_type
POLYTOPE, SPHERE, CONE, CAPSULE, CYLINDER, POLYGON = range(6)
# enum dcol_status
OK, MAXITER, UNSUPPORTED, NOT_PD, NONFINITE, TOO_LARGE = range(6)
# enum dcol_flags
GRAD_FD, GRAD_ENVELOPE, CONTACT, CASE4, GRAD_IMPLICIT, NO_GATHER = 1, 2, 4, 8, 16, 32
GRAD_ANY = GRAD_FD | GRAD_ENVELOPE | GRAD_IMPLICIT
# enum dcol_plan_options
PLAN_CASE4, PLAN_NO_FUSE, PLAN_SUSPEND = 1, 2, 4
SUCCESS, ERR_ARG, ERR_HIP, ERR_NOMEM = 0, -1, -2, -3
ABI_VERSION = 4
PAIR_PLANS_MAX = 64   # DCOL_PAIR_PLANS_MAX


class DcolLibraryError(RuntimeError):
    pass


class ShapeDesc(ctypes.Structure):
    """struct dcol_shape_desc"""
    _fields_ = [("type", c_int32), ("nh", c_int32), ("A", POINTER(c_double)), ("b", POINTER(c_double)),
                ("R", c_double), ("L", c_double), ("H", c_double), ("beta", c_double),
                ("r_offset", c_double * 3), ("Q_offset", c_double * 9)]


# name -> (restype, argtypes); must match include/dcol.h exactly (checked by tests/test_cabi.py)
SIGNATURES = {
    "dcol_abi_version": (c_int, []),
    "dcol_status_string": (c_char_p, [c_int32]),
    "dcol_last_error": (c_char_p, []),
    "dcol_device_count": (c_int, [POINTER(c_int32)]),
    "dcol_table_create": (c_int, [POINTER(ShapeDesc), c_int32, c_int32, POINTER(c_void_p)]),
    "dcol_table_destroy": (c_int, [c_void_p]),
    "dcol_table_size": (c_int, [c_void_p, POINTER(c_int32)]),
    "dcol_pair_dims": (c_int, [c_void_p, c_int32, c_int32, POINTER(c_int32), POINTER(c_int32),
                               POINTER(c_int32), POINTER(c_int32)]),
    "dcol_plan_create": (c_int, [c_void_p, c_int64, c_void_p, c_void_p, POINTER(c_void_p)]),
    "dcol_plan_create_ex": (c_int, [c_void_p, c_int64, c_void_p, c_void_p, c_int32, POINTER(c_void_p)]),
    "dcol_plan_destroy": (c_int, [c_void_p]),
    "dcol_plan_num_launches": (c_int, [c_void_p, POINTER(c_int32)]),
    "dcol_plan_num_streams": (c_int, [c_void_p, POINTER(c_int32)]),
    "dcol_plan_launch_form": (c_int, [c_void_p, POINTER(c_int32)]),
    "dcol_plan_num_buckets": (c_int, [c_void_p, POINTER(c_int32)]),
    "dcol_plan_bucket": (c_int, [c_void_p, c_int32, POINTER(c_int32), POINTER(c_int64)]),
    "dcol_plan_suspended": (c_int, [c_void_p, POINTER(c_int64)]),
    "dcol_plan_run": (c_int, [c_void_p, c_void_p, c_void_p, c_double, c_int32, c_int32, c_void_p, c_void_p,
                              c_void_p, c_void_p, c_void_p, c_void_p]),
    "dcol_prox_batch_host": (c_int, [c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_void_p, c_double,
                                     c_int32, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "dcol_prox_pair": (c_int, [c_void_p, c_int32, c_int32, c_void_p, c_void_p, c_double, c_int32, c_int32, c_void_p,
                               c_void_p, c_void_p, c_void_p, c_void_p]),
    "dcol_table_pair_plans": (c_int, [c_void_p, POINTER(c_int32)]),
    "dcol_table_pair_stats": (c_int, [c_void_p, POINTER(c_int64), POINTER(c_int64), POINTER(c_int64),
                                      POINTER(c_double), POINTER(c_double), POINTER(c_int32)]),
    "dcol_debug_pair_stamps": (c_int, [c_void_p, c_void_p]),
    "dcol_table_stop_pair_server": (c_int, [c_void_p]),
    "dcol_table_pair_server_running": (c_int, [c_void_p, POINTER(c_int32)]),
    "dcol_shutdown": (c_int, []),
    "dcol_comm_unique_id": (c_int, [c_void_p]),
    "dcol_comm_create": (c_int, [c_void_p, c_int32, c_int32, c_int32, POINTER(c_void_p)]),
    "dcol_comm_destroy": (c_int, [c_void_p]),
    "dcol_prox_batch_multi_gpu": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_double, c_int32, c_int32,
                                          c_int64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                          c_void_p]),
    "dcol_comm_all_gather": (c_int, [c_void_p, c_int64, c_void_p, c_void_p]),
}
COMM_ID_BYTES = 128

_lib = None
_load_error = None


def load(path: str | None = None):
    """Load (once) and return the ctypes library; raise DcolLibraryError if unavailable."""
    global _lib, _load_error
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        _load_error = f"{p} not found: build it with `make -C {os.path.join(PKG_ROOT, 'csrc')}` (or __graft_entry__.build())"
        raise DcolLibraryError(_load_error)
    try:
        lib = ctypes.CDLL(p)
    except OSError as e:  # pragma: no cover - environment specific
        _load_error = f"cannot load {p}: {e}"
        raise DcolLibraryError(_load_error) from e
    # the version first: a stale library lacks some of the entry points bound below, and
    # must fail with this message rather than a bare AttributeError from getattr
    try:
        ver_fn = lib.dcol_abi_version
    except AttributeError as e:
        raise DcolLibraryError(f"{p}: no dcol_abi_version export (not a libdcol build)") from e
    ver_fn.restype = ctypes.c_int
    ver_fn.argtypes = []
    if ver_fn() != ABI_VERSION:
        raise DcolLibraryError(f"{p}: ABI version {ver_fn()} != {ABI_VERSION} (rebuild: make -C "
                               f"{os.path.join(PKG_ROOT, 'csrc')})")
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if path is None:
        _lib = lib
        # stop every resident pair server before interpreter teardown: Table.__del__ (which
        # would stop its table's) is not guaranteed to run at exit.  The library's own exit
        # handler does the same later; this one runs while Python still owns its threads.
        atexit.register(_shutdown)
    return lib


def _shutdown():
    if _lib is not None:
        _lib.dcol_shutdown()


def check(rc: int, what: str = ""):
    if rc != SUCCESS:
        msg = load().dcol_last_error().decode(errors="replace")
        raise DcolLibraryError(f"{what}: error {rc}: {msg}")


def status_string(code: int) -> str:
    return load().dcol_status_string(int(code)).decode()


def device_count() -> int:
    n = c_int32(0)
    check(load().dcol_device_count(ctypes.byref(n)), "dcol_device_count")
    return int(n.value)


_hip = None


def host_device_pointer(ptr: int):
    """Device address of a pinned host allocation (hipHostGetDevicePointer), or None when the
    allocation is not mapped into the device's address space (the caller then stages
    through copies instead)."""
    global _hip
    if _hip is None:
        try:
            _hip = ctypes.CDLL("libamdhip64.so")
            _hip.hipHostGetDevicePointer.restype = c_int
            _hip.hipHostGetDevicePointer.argtypes = [POINTER(c_void_p), c_void_p, ctypes.c_uint]
        except OSError:
            _hip = False
    if not _hip:
        return None
    out = c_void_p()
    if _hip.hipHostGetDevicePointer(ctypes.byref(out), c_void_p(ptr), 0) != 0 or not out.value:
        return None
    return out.value
