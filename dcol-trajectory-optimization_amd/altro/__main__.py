"""python -m altro --system {piano_mover,quadrotor,coneThroughWall} [--quiet]

Counterpart of the reference's main.py (without the matplotlib scene rendering): runs the
batched ALTRO on the GPU and prints iterations, wall time and the proximity share."""
import argparse
import json
import logging

from . import solve, systems


def main():
    ap = argparse.ArgumentParser(description="Batched ALTRO over the GPU proximity engine")
    ap.add_argument("--system", required=True, choices=["piano_mover", "quadrotor", "coneThroughWall"])
    ap.add_argument("--quiet", action="store_true")
    args = ap.parse_args()
    logging.basicConfig(level=logging.INFO, format="%(levelname)s - %(message)s")
    params, X, U = systems.initialize(args.system)
    r = solve(params, X, U, verbose=not args.quiet)
    print(json.dumps({"system": args.system, "converged": r.converged, "iterations": r.iterations,
                      "wall_s": round(r.wall_s, 4), "setup_s": round(r.setup_s, 4), "ms_per_iter": round(r.ms_per_iter, 3),
                      "prox_s": round(r.prox_s, 4), "prox_batches": r.prox_batches, "prox_pairs": r.prox_pairs,
                      "J_final": r.J[-1] if r.J else None}))


if __name__ == "__main__":
    main()
