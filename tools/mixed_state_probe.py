#!/usr/bin/env python3
"""Diagnostic: the mixed 1M solve time (HIP events, the plan's launch only) in a fresh
process after different prior work in the same process (bench.py's default line measures
configs[4] after the polytope section).  Usage: python3 tools/mixed_state_probe.py MODE
  fresh | poly_plan (engine + plan + buffers of the 100k section, no runs) | poly_run (its
  launches) | e2e (its end_to_end section) | pinned (a 100 MB pinned host buffer) |
  pool_first (torch's stream pool created before the plan's side streams)"""
import os
import sys
import time

import numpy as np

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [REPO, os.path.join(REPO, "dcol-trajectory-optimization_amd")]
import bench  # noqa: E402


def mixed_solve_ms(dev):
    import torch
    from dcol_amd import Engine, alloc_outputs, spec_from_arrays
    tab = bench.mixed_table()
    s1, s2, p1, p2 = bench.mixed_pairs(tab, 1_000_000, seed=0)
    eng = Engine(device=0)
    ids = np.array([eng.register(spec_from_arrays(tab, k)) for k in range(len(tab["type"]))], np.int32)
    plan = eng.plan(ids[s1], ids[s2])
    d1 = torch.from_numpy(np.ascontiguousarray(p1.T)).to(dev)
    d2 = torch.from_numpy(np.ascontiguousarray(p2.T)).to(dev)
    out = alloc_outputs(len(s1), dev, want_grad=True, want_contact=False)
    st = torch.cuda.current_stream(dev)
    run = plan.bind(d1, d2, out, grad="fd", contact=False, stream=st)
    for _ in range(30):
        run()
    torch.cuda.synchronize(dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(10)]
    for a, b in ev:
        a.record(st)
        run()
        b.record(st)
    torch.cuda.synchronize(dev)
    return float(np.median([a.elapsed_time(b) for a, b in ev]))


def main():
    import torch
    mode = sys.argv[1]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    if mode != "fresh":
        from dcol_amd import Engine, alloc_outputs, spec_from_arrays
        if mode == "pool_first":
            torch.cuda.Stream(dev)
        elif mode == "pinned":
            keep = torch.empty(100_000_000 // 8, dtype=torch.float64).pin_memory()   # noqa: F841
        else:
            tab = bench.shape_table()
            s1, s2, p1, p2 = bench.pairs(100_000, len(tab["type"]), seed=1000)
            eng = Engine(device=0)
            ids = np.array([eng.register(spec_from_arrays(tab, k)) for k in range(len(tab["type"]))], np.int32)
            plan = eng.plan(ids[s1], ids[s2])
            pose1 = torch.from_numpy(np.ascontiguousarray(p1.T)).to(dev)
            pose2 = torch.from_numpy(np.ascontiguousarray(p2.T)).to(dev)
            out = alloc_outputs(100_000, dev, want_grad=True, want_contact=False)
            step = plan.bind(pose1, pose2, out, grad="fd", contact=False, stream=torch.cuda.current_stream(dev))
            if mode == "poly_run":
                for _ in range(50):
                    step()
                torch.cuda.synchronize(dev)
            if mode == "e2e":
                class A:
                    grad = "fd"
                bench.end_to_end(A, eng, ids, s1, s2, p1, p2, pose1, pose2, out, step, dev, reps=3)
    t0 = time.perf_counter()
    ms = mixed_solve_ms(dev)
    print(f"{mode}: mixed 1M solve {ms:.4f} ms ({1e6 / (ms * 1e-3):.3e} pair-solves/s), setup+run {time.perf_counter() - t0:.1f} s",
          flush=True)


if __name__ == "__main__":
    main()
