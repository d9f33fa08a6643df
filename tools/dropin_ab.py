#!/usr/bin/env python3
"""Drop-in per-call latency with and without dcol_prox_pair's one-pair server: bench.py's
`dropin` section (the quadrotor hallway, one call per pair, the reference's calling
pattern) run alternately under DCOL_PAIR_SERVER=1 and =0 (the library reads it per call),
plus the served / launched counters of the engine's table.
Usage: python3 tools/dropin_ab.py [--rounds 3]
"""
import argparse
import json
import os
import sys

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [REPO, os.path.join(REPO, "dcol-trajectory-optimization_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    import bench
    from dcol_amd.engine import default_engine
    for r in range(args.rounds):
        for server in ("1", "0"):
            os.environ["DCOL_PAIR_SERVER"] = server
            s0 = default_engine().pair_stats()
            out = bench.dropin_section()
            s1 = default_engine().pair_stats()
            n = s1["served"] - s0["served"]
            row = {"round": r, "server": server,
                   "mrp_us": round(out["proximity_mrp"]["us_per_call"], 2),
                   "grad_us": round(out["proximity_gradient"]["us_per_call"], 2),
                   "served": n, "launched": s1["launched"] - s0["launched"]}
            if n:   # device time from request seen to answer stored, and the clock it ran at
                us = s1["server_solve_us"] - s0["server_solve_us"]
                cyc = s1["server_solve_cycles"] - s0["server_solve_cycles"]
                row["device_us_per_call"] = round(us / n, 2)
                row["clock_ghz"] = round(cyc / us / 1e3, 3)
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
