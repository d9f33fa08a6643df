#!/usr/bin/env python3
"""Drop-in calls alternating proximity_mrp / proximity_gradient call by call (the pair
server's flags differ between the two, so it restarts at every switch) against the phase
pattern (all mrp calls, then all gradient calls), with and without the server.
Usage: python3 tools/alternate_probe.py"""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [REPO, os.path.join(REPO, "dcol-trajectory-optimization_amd")]


def main():
    from altro import systems
    from proximity.proximity import proximity_mrp
    from proximity.proximity_gradient import proximity_gradient
    params, X, U = systems.initialize("quadrotor")
    vic, obs = params["P_vic"], params["P_obs"]
    Xr = np.asarray(params["Xref"], dtype=np.float64).reshape(-1, int(params["nx"]))
    for fn in (proximity_mrp, proximity_gradient):
        for o in obs:
            fn(vic, o)
    for server in ("1", "0", "1", "0"):
        os.environ["DCOL_PAIR_SERVER"] = server
        for pattern in ("alternate", "phases"):
            t0 = time.perf_counter()
            n = 0
            if pattern == "alternate":
                for x in Xr[:50]:
                    vic.r, vic.p = np.array(x[0:3]), np.array(x[6:9])
                    for o in obs:
                        proximity_mrp(vic, o)
                        proximity_gradient(vic, o)
                        n += 2
            else:
                for fn in (proximity_mrp, proximity_gradient):
                    for x in Xr[:50]:
                        vic.r, vic.p = np.array(x[0:3]), np.array(x[6:9])
                        for o in obs:
                            fn(vic, o)
                            n += 1
            dt = time.perf_counter() - t0
            print(json.dumps({"server": server, "pattern": pattern, "us_per_call": round(1e6 * dt / n, 2)}), flush=True)


if __name__ == "__main__":
    main()
