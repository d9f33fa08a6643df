#!/usr/bin/env python3
"""Latency anatomy of one ALTRO phase batch (ObstacleField.evaluate) per reference scene:
wall time of the whole evaluate() call (H2D poses, fan-out launches, D2H, sync), of the
launch alone (back-to-back, same stream), and of one launch + sync.  Run it under
`rocprofv3 --kernel-trace` to see the per-variant kernel durations and the gaps.
DCOL_ALTRO_PHASE=zero_copy|graph|eager selects how a phase reaches the GPU (constraints.py).
Usage: python3 tools/scene_latency.py [reps]"""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(REPO, "dcol-trajectory-optimization_amd"), REPO]


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    import torch
    from altro import systems
    from altro.constraints import ObstacleField
    for name in ("quadrotor", "coneThroughWall", "piano_mover"):
        params, X, U = systems.initialize(name)
        mod = systems.get(name)
        f = ObstacleField(params["P_vic"], params["P_obs"], params["N"])
        P = mod.victim_poses(params, np.asarray(params["Xref"], dtype=np.float64))
        f.evaluate(P, True)
        torch.cuda.synchronize()
        t = {}
        t0 = time.perf_counter()
        for _ in range(reps):
            f.evaluate(P, True)
        t["evaluate_grad_ms"] = 1e3 * (time.perf_counter() - t0) / reps
        t0 = time.perf_counter()
        for _ in range(reps):
            f.evaluate(P, False)
        t["evaluate_alpha_ms"] = 1e3 * (time.perf_counter() - t0) / reps
        t0 = time.perf_counter()
        for _ in range(reps):
            f._launch[True]()
            f.stream.synchronize()
        t["launch_sync_ms"] = 1e3 * (time.perf_counter() - t0) / reps
        t0 = time.perf_counter()
        for _ in range(reps):
            f._launch[True]()
        torch.cuda.synchronize()
        t["launch_pipelined_ms"] = 1e3 * (time.perf_counter() - t0) / reps
        t0 = time.perf_counter()
        for _ in range(reps):
            f._launch[True]()
        t["launch_host_ms"] = 1e3 * (time.perf_counter() - t0) / reps
        torch.cuda.synchronize()
        print(json.dumps({"scene": name, "mode": f.mode, "pairs": f.B, "launches": f.plan.num_launches,
                          **{k: round(v, 4) for k, v in t.items()}}), flush=True)


if __name__ == "__main__":
    main()
