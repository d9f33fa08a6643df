#!/usr/bin/env python3
"""DPP-source check: runs the golden vectors, the 1M mixed workload
and the 100k benchmark batch through the diagnostic build lib_check/libdcol.so (make -C
dcol-trajectory-optimization_amd/csrc check-exec), in which every DPP lane read whose
source lane is inactive increments a counter (dcol_device.hpp dpp_check), and prints the
counts.  Zero everywhere = no reduction ever reads a register its partner lane did not
write, on any of these workloads, under any of the kernels they reach (per-variant,
fused, row-partitioned).  Usage: python3 tools/check_exec.py
"""
import ctypes
import glob
import json
import os
import sys

import numpy as np

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
PKG = os.path.join(REPO, "dcol-trajectory-optimization_amd")
LIB = os.path.join(PKG, "lib_check", "libdcol.so")
os.environ["DCOL_LIB"] = LIB
sys.path[:0] = [PKG, REPO, os.path.join(REPO, "tests")]


def main():
    import bench
    from conftest import load_golden
    from dcol_amd import Engine, _lib, spec_from_arrays
    lib = _lib.load()
    fn = lib.dcol_debug_exec_violations
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.c_int32]
    v = ctypes.c_uint64()

    def count(reset=True):
        _lib.check(fn(ctypes.byref(v), 1 if reset else 0), "dcol_debug_exec_violations")
        return int(v.value)

    count()
    out = {}
    # positive control: a kernel whose 2-lane sums read from inactive partner lanes (one wave,
    # 32 reads) -- the detector must count them
    st = lib.dcol_debug_exec_selftest
    st.restype = ctypes.c_int
    st.argtypes = [ctypes.POINTER(ctypes.c_uint64)]
    _lib.check(st(ctypes.byref(v)), "dcol_debug_exec_selftest")
    out["positive_control_expected_32"] = int(v.value)
    count()
    eng = Engine(device=0)
    for path in sorted(glob.glob(os.path.join(REPO, "tests", "golden", "*.npz"))):
        d = load_golden(path)
        if "s1" not in d:
            continue
        ids = np.array([eng.register(spec_from_arrays(d, k)) for k in range(len(d["type"]))], np.int32)
        for grad in ("fd", "envelope", "implicit"):
            eng.solve_host(ids[d["s1"]], ids[d["s2"]], d["pose1"], d["pose2"], tol=float(d["tol"]), grad=grad,
                           contact=True)
        out[os.path.basename(path)] = {"pairs": int(len(d["s1"])), "violations": count()}
    tab = bench.mixed_table()
    s1, s2, p1, p2 = bench.mixed_pairs(tab, 1_000_000, seed=0)
    ids = np.array([eng.register(spec_from_arrays(tab, k)) for k in range(len(tab["type"]))], np.int32)
    eng.solve_host(ids[s1], ids[s2], p1, p2, grad="fd", contact=True)
    out["mixed1m"] = {"pairs": 1_000_000, "violations": count()}
    tab = bench.shape_table()
    s1, s2, p1, p2 = bench.pairs(100_000, len(tab["type"]), seed=1000)
    ids = np.array([eng.register(spec_from_arrays(tab, k)) for k in range(len(tab["type"]))], np.int32)
    eng.solve_host(ids[s1], ids[s2], p1, p2, grad="fd", contact=True)
    out["poly100k"] = {"pairs": 100_000, "violations": count()}
    out["total"] = sum(r["violations"] for r in out.values() if isinstance(r, dict))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
