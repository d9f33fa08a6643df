"""ctypes wrapper of the C oracle (oracle/dcol_oracle.c).  TEST INFRASTRUCTURE ONLY.

run_batch() has the same inputs/outputs as oracle.dcol_oracle.run_batch (shape table in
the tests/golden array layout), parallelised with OpenMP over `threads` host cores."""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "libdcol_oracle.so")
_lib = None


def build():
    subprocess.run(["make", "-C", HERE, "-s"], check=True)


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        _lib = ctypes.CDLL(LIB)
        _lib.dcol_oracle_batch.restype = ctypes.c_int
    return _lib


def _p(a):
    return ctypes.c_void_p(a.ctypes.data)


def run_batch(tab, s1, s2, pose1, pose2, tol=1e-6, want_grad=True, threads=1):
    lib = load()
    B = len(s1)
    c = lambda a, dt: np.ascontiguousarray(a, dtype=dt)  # noqa: E731
    t = {k: c(tab[k], np.int32) for k in ("type", "nh", "A_off")}
    f = {k: c(tab[k], np.float64) for k in ("A_pool", "b_pool", "params", "r_offset", "Q_offset")}
    if f["A_pool"].size == 0:
        f["A_pool"] = np.zeros((1, 3))
        f["b_pool"] = np.zeros(1)
    s1, s2 = c(s1, np.int32), c(s2, np.int32)
    p1, p2 = c(pose1, np.float64), c(pose2, np.float64)
    out = dict(alpha=np.empty(B), contact=np.empty((B, 3)), grad=np.empty((B, 12)),
               iters=np.empty(B, np.int32), status=np.empty(B, np.int32))
    lib.dcol_oracle_batch(ctypes.c_int32(len(t["type"])), _p(t["type"]), _p(t["nh"]), _p(t["A_off"]),
                          _p(f["A_pool"]), _p(f["b_pool"]), _p(f["params"]), _p(f["r_offset"]), _p(f["Q_offset"]),
                          ctypes.c_int64(B), _p(s1), _p(s2), _p(p1), _p(p2), ctypes.c_double(tol),
                          ctypes.c_int32(int(want_grad)), ctypes.c_int32(int(threads)), _p(out["alpha"]),
                          _p(out["contact"]), _p(out["grad"]), _p(out["iters"]), _p(out["status"]))
    return out


OPC_LIB = os.path.join(HERE, "build", "libdcol_oracle_opcount.so")


def op_counts(tab, s1, s2, pose1, pose2, tol=1e-6):
    """FP64 operation counts per pair of the C restatement (dcol_oracle_opcount.cpp: each
    +, -, *, / and sqrt the reference's algorithm executes = 1), split by phase:
    dict(assembly, pdip, grad, iters, status), int64 [B] each (iters/status int32)."""
    if not os.path.exists(OPC_LIB):
        build()
    lib = ctypes.CDLL(OPC_LIB)
    B = len(s1)
    c = lambda a, dt: np.ascontiguousarray(a, dtype=dt)  # noqa: E731
    t = {k: c(tab[k], np.int32) for k in ("type", "nh", "A_off")}
    f = {k: c(tab[k], np.float64) for k in ("A_pool", "b_pool", "params", "r_offset", "Q_offset")}
    if f["A_pool"].size == 0:
        f["A_pool"] = np.zeros((1, 3))
        f["b_pool"] = np.zeros(1)
    s1, s2 = c(s1, np.int32), c(s2, np.int32)
    p1, p2 = c(pose1, np.float64), c(pose2, np.float64)
    out = dict(assembly=np.empty(B, np.int64), pdip=np.empty(B, np.int64), grad=np.empty(B, np.int64),
               iters=np.empty(B, np.int32), status=np.empty(B, np.int32))
    rc = lib.dcol_opcount_batch(_p(t["type"]), _p(t["nh"]), _p(t["A_off"]), _p(f["A_pool"]), _p(f["b_pool"]),
                                _p(f["params"]), _p(f["r_offset"]), _p(f["Q_offset"]), ctypes.c_int64(B), _p(s1),
                                _p(s2), _p(p1), _p(p2), ctypes.c_double(tol), _p(out["assembly"]), _p(out["pdip"]),
                                _p(out["grad"]), _p(out["iters"]), _p(out["status"]))
    assert rc == 0
    return out
