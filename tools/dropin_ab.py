#!/usr/bin/env python3
"""Drop-in per-call latency with and without dcol_prox_pair's one-pair server: the quadrotor
hallway sweep of bench.py's `dropin` section (100 knots x 11 obstacles, one call per pair,
P_vic.r / .p overwritten per knot), one call kind at a time, alternately under
DCOL_PAIR_SERVER=1 and =0 (the library reads it per call).  Per sweep: host us per call,
the served / launched counters, the server's device request-to-answer time, the clock it
ran at and the XCD it sat on (dcol_table_pair_stats).
Usage: python3 tools/dropin_ab.py [--rounds 3] [--reps 3]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [REPO, os.path.join(REPO, "dcol-trajectory-optimization_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    from altro import systems
    from dcol_amd.engine import default_engine
    from proximity.proximity import proximity_mrp
    from proximity.proximity_gradient import proximity_gradient
    params, X, U = systems.initialize("quadrotor")
    vic, obs = params["P_vic"], params["P_obs"]
    Xr = np.asarray(params["Xref"], dtype=np.float64).reshape(-1, int(params["nx"]))
    eng = default_engine()
    for fn in (proximity_mrp, proximity_gradient):   # shapes registered, plans built
        for o in obs:
            fn(vic, o)
    for r in range(args.rounds):
        for server in ("1", "0"):
            os.environ["DCOL_PAIR_SERVER"] = server
            for name, fn in (("mrp", proximity_mrp), ("grad", proximity_gradient)):
                fn(vic, obs[0])                       # (re)start the server for this call kind
                s0 = eng.pair_stats()
                best = None
                for _ in range(args.reps):
                    t0 = time.perf_counter()
                    for x in Xr:
                        vic.r = np.array(x[0:3])
                        vic.p = np.array(x[6:9])
                        for o in obs:
                            fn(vic, o)
                    dt = time.perf_counter() - t0
                    best = dt if best is None else min(best, dt)
                s1 = eng.pair_stats()
                n = s1["served"] - s0["served"]
                row = {"round": r, "server": server, "call": name, "us_per_call": round(1e6 * best / (len(Xr) * len(obs)), 2),
                       "served": n, "launched": s1["launched"] - s0["launched"]}
                if n:
                    us = s1["server_solve_us"] - s0["server_solve_us"]
                    cyc = s1["server_solve_cycles"] - s0["server_solve_cycles"]
                    row["device_us_per_call"] = round(us / n, 2)
                    row["clock_ghz"] = round(cyc / us / 1e3, 3)
                    row["server_xcd"] = s1["server_xcd"]
                print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
