#!/usr/bin/env python3
"""Per-call device time of the one-pair server (dcol_table_pair_stats around every call),
per obstacle of the quadrotor hallway, in two call orders:
  mixed : the reference's order -- every obstacle at every knot (11 different pairs in turn,
          6 kernel variants: the server's solver copies alternate call by call),
  single: all knots against one obstacle, then the next obstacle (one variant at a time).
The same calls in both orders; a per-obstacle gap points at per-call costs that depend on
what ran before (instruction cache, L2), not at the solve itself.
Usage: python3 tools/dropin_percall.py [--grad]"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [REPO, os.path.join(REPO, "dcol-trajectory-optimization_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grad", action="store_true")
    args = ap.parse_args()
    from altro import systems
    from dcol_amd.engine import default_engine
    params, X, U = systems.initialize("quadrotor")
    vic, obs = params["P_vic"], params["P_obs"]
    Xr = np.asarray(params["Xref"], dtype=np.float64).reshape(-1, int(params["nx"]))
    eng = default_engine()
    grad = "fd" if args.grad else None
    for o in obs:
        eng.solve_pair(vic, o, grad=grad)

    def call(x, o):
        vic.r = np.array(x[0:3])
        vic.p = np.array(x[6:9])
        s0 = eng.pair_stats()["server_solve_us"]
        eng.solve_pair(vic, o, grad=grad)
        return eng.pair_stats()["server_solve_us"] - s0

    for order in ("mixed", "single", "mixed", "single"):
        dev = np.zeros((len(obs), len(Xr)))
        if order == "mixed":
            for k, x in enumerate(Xr):
                for j, o in enumerate(obs):
                    dev[j, k] = call(x, o)
        else:
            for j, o in enumerate(obs):
                for k, x in enumerate(Xr):
                    dev[j, k] = call(x, o)
        print(json.dumps({"order": order, "grad": bool(args.grad), "mean_us": round(float(dev.mean()), 2),
                          "per_obstacle_us": [round(float(v), 2) for v in dev.mean(axis=1)],
                          "obstacles": [type(o).__name__ for o in obs]}), flush=True)


if __name__ == "__main__":
    main()
