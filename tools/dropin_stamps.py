#!/usr/bin/env python3
"""Where a drop-in call's device time goes, request by request (the stamps build of the
library: `make -C dcol-trajectory-optimization_amd/csrc stamps`, DCOL_LIB=.../lib_stamps/libdcol.so):
the quadrotor hallway sweep of bench.py's `dropin` section (100 knots x 11 obstacles, one call
per pair), and for every call answered by the one-pair server its shader-clock stamps
(dcol_debug_pair_stamps): request seen -> solve start -> frames (the poses read from mapped
host memory, the DCMs) -> assembly (shape records / rows) -> initialise -> PDIP loop ->
gradient (re-reads the poses) -> answer released.  Prints per sweep and call kind the
median cycles per phase, the Newton iterations, the device time and the server's XCD.
Usage: DCOL_LIB=<lib_stamps> python3 tools/dropin_stamps.py [--sweeps 3] [--label x]"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(REPO, "dcol-trajectory-optimization_amd"), REPO]

PHASES = ("req_to_start", "frames", "assembly", "initialise", "pdip_loop", "gradient", "stores_answer")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sweeps", type=int, default=3)
    ap.add_argument("--label", default="")
    a = ap.parse_args()
    from altro import systems
    from dcol_amd import _lib
    from dcol_amd.engine import default_engine
    params, X, U = systems.initialize("quadrotor")
    vic, obs = params["P_vic"], params["P_obs"]
    Xr = np.asarray(params["Xref"], dtype=np.float64).reshape(-1, int(params["nx"]))
    eng = default_engine()
    lib = _lib.load()
    buf = (ctypes.c_uint64 * 16)()
    for grad in (None, "fd"):
        for o in obs:
            eng.solve_pair(vic, o, grad=grad)
    for sw in range(a.sweeps):
        for kind, grad in (("mrp", None), ("grad", "fd")):
            rows, its, names = [], [], []
            s0 = eng.pair_stats()
            t0 = time.perf_counter()
            for x in Xr:
                vic.r = np.array(x[0:3])
                vic.p = np.array(x[6:9])
                for o in obs:
                    r = eng.solve_pair(vic, o, grad=grad, contact=(grad is None))
                    _lib.check(lib.dcol_debug_pair_stamps(eng.table.handle, buf), "dcol_debug_pair_stamps")
                    s = [int(v) for v in buf]
                    rows.append([s[0] - s[6], s[1] - s[0], s[2] - s[1], s[3] - s[2], s[4] - s[3], s[5] - s[4],
                                 s[7] - s[5]])
                    its.append(r[3])
                    names.append(type(o).__name__)
            wall = (time.perf_counter() - t0) / len(rows)
            s1 = eng.pair_stats()
            n = s1["served"] - s0["served"]
            R = np.array(rows, dtype=np.float64)
            out = {"label": a.label, "sweep": sw, "kind": kind, "calls": len(rows), "served": n,
                   "us_per_call": 1e6 * wall,
                   "device_us_per_call": (s1["server_solve_us"] - s0["server_solve_us"]) / max(n, 1),
                   "clock_ghz": (s1["server_solve_cycles"] - s0["server_solve_cycles"])
                   / max(s1["server_solve_us"] - s0["server_solve_us"], 1e-9) / 1e3,
                   "xcd": s1["server_xcd"], "iters_mean": float(np.mean(its)),
                   "median_cycles": dict(zip(PHASES, np.median(R, axis=0).round(0).tolist())),
                   "mean_cycles": dict(zip(PHASES, R.mean(axis=0).round(0).tolist())),
                   "loop_cycles_per_iteration": float(np.median(R[:, 4] / np.maximum(np.array(its), 1)))}
            by = {}
            for nm in sorted(set(names)):
                m = np.array([q == nm for q in names])
                by[nm] = {"calls": int(m.sum()), "total_cycles": float(np.median(R[m].sum(axis=1))),
                          "loop": float(np.median(R[m, 4])), "iters": float(np.mean(np.array(its)[m]))}
            out["by_obstacle"] = by
            print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
