#!/usr/bin/env python3
"""ALTRO wall-clock per iteration with a host-side breakdown: every native call the driver
makes (altro._native.*) and the time blocked in the proximity evaluator are timed by
wrapping them; best of --reps runs per system.
Usage: python3 tools/altro_profile.py [quadrotor coneThroughWall piano_mover] [--reps 3]"""
import argparse
import json
import logging
import os
import sys
import time

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(REPO, "dcol-trajectory-optimization_amd"), REPO]

from altro import driver, solve, systems  # noqa: E402

TIMED = ("jacobians", "backward", "stage_terms", "rollout", "rollouts", "cost", "victim_poses", "constraint_jacobian",
         "backward_pass", "trial")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("systems", nargs="*", default=["quadrotor", "coneThroughWall", "piano_mover"])
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    logging.getLogger("altro").setLevel(logging.WARNING)
    acc = {}
    nat = driver._native
    orig = {n: getattr(nat, n) for n in TIMED}

    def wrap(n):
        f = orig[n]

        def g(*a, **k):
            t0 = time.perf_counter()
            try:
                return f(*a, **k)
            finally:
                acc[n] = acc.get(n, 0.0) + time.perf_counter() - t0
        return g
    for n in TIMED:
        setattr(nat, n, wrap(n))
    for name in args.systems:
        best = None
        for _ in range(args.reps):
            params, X, U = systems.initialize(name)
            acc.clear()
            r = solve(params, X, U, verbose=False)
            if best is None or r.wall_s < best[0].wall_s:
                best = (r, dict(acc))
        r, parts = best
        it = max(r.iterations, 1)
        out = {"system": name, "iterations": r.iterations, "ms_per_iter": round(r.ms_per_iter, 4),
               "prox_blocked_ms_per_iter": round(1e3 * r.prox_s / it, 4), "prox_batches": r.prox_batches}
        out.update({f"{k}_ms_per_iter": round(1e3 * v / it, 4) for k, v in sorted(parts.items())})
        out["other_host_ms_per_iter"] = round(r.ms_per_iter - 1e3 * (r.prox_s + sum(parts.values())) / it, 4)
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
