#!/usr/bin/env python3
"""Listing order of configs[4]'s 1M mixed pairing on one GPU: the given (random) listing
against dcol_amd.cost_order of one solve's iteration counts, K steps back to back (HIP
events), at the same poses every step and at drifting poses (a random walk from the mixed
poses, r + N(0, sr), p + N(0, sp) per step, a ring walked forth and back).  A bucketed plan
already reads its pairs through a permutation, so the re-listing changes only which pairs
share a wave.  Outputs of the last step compared bitwise (un-permuted).

  python3 tools/mixed_order.py [--steps 30] [--sr 0.02] [--sp 0.01] [--ring 8]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [ROOT, os.path.join(ROOT, "dcol-trajectory-optimization_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--sr", type=float, default=0.02)
    ap.add_argument("--sp", type=float, default=0.01)
    ap.add_argument("--ring", type=int, default=8)
    a = ap.parse_args()
    os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")
    import torch

    import bench
    from dcol_amd import Engine, alloc_outputs, cost_order, spec_from_arrays
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    eng = Engine(device=0)
    stream = torch.cuda.current_stream(dev)
    mt = bench.mixed_table()
    ids = np.array([eng.register(spec_from_arrays(mt, k)) for k in range(len(mt["type"]))], np.int32)
    B = 1_000_000
    s1, s2, p1, p2 = bench.mixed_pairs(mt, B, seed=0)
    rng = np.random.default_rng(9)
    walk = [(p1, p2)]
    for _ in range(a.ring - 1):
        q1, q2 = walk[-1][0].copy(), walk[-1][1].copy()
        for q in (q1, q2):
            q[:, :3] += rng.normal(0, a.sr, (B, 3))
            q[:, 3:] += rng.normal(0, a.sp, (B, 3))
        walk.append((q1, q2))
    seq = list(range(a.ring)) + list(range(a.ring - 2, 0, -1))
    first, outs = None, {}
    for name in ("given", "cost"):
        order = np.arange(B) if name == "given" else cost_order(first)
        plan = eng.plan(ids[s1[order]], ids[s2[order]], cache=False)
        dp = [(torch.from_numpy(np.ascontiguousarray(x[order].T)).to(dev),
               torch.from_numpy(np.ascontiguousarray(y[order].T)).to(dev)) for x, y in walk]
        out = alloc_outputs(B, dev, want_grad=True, want_contact=False)
        runs = [plan.bind(d1, d2, out, grad="fd", contact=False, stream=stream) for d1, d2 in dp]
        runs[0]()
        torch.cuda.synchronize(dev)
        if first is None:
            first = out["iters"].cpu().numpy()
        bench.clock_settle(runs[0], stream, dev, None, 30.0)
        for mode in ("same_poses", "drifting_poses"):
            for k in range(5):
                runs[0 if mode == "same_poses" else seq[k % len(seq)]]()
            torch.cuda.synchronize(dev)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for k in range(a.steps):
                runs[0 if mode == "same_poses" else seq[(5 + k) % len(seq)]]()
            e1.record(stream)
            torch.cuda.synchronize(dev)
            ms = e0.elapsed_time(e1) / a.steps
            print(json.dumps({"order": name, "poses": mode, "ms_per_step": ms, "pair_solves_per_s": B / (ms * 1e-3),
                              "launches": plan.num_launches, "form": plan.launch_form}), flush=True)
        runs[0]()
        torch.cuda.synchronize(dev)
        inv = np.empty(B, np.int64)
        inv[order] = np.arange(B)
        outs[name] = {k: v.cpu().numpy()[..., inv] for k, v in out.items()}
        del runs, dp, out, plan
    eq = all(np.array_equal(outs["given"][k].view(np.int64) if outs["given"][k].dtype == np.float64 else outs["given"][k],
                            outs["cost"][k].view(np.int64) if outs["cost"][k].dtype == np.float64 else outs["cost"][k])
             for k in outs["given"])
    print(json.dumps({"bitwise_equal_first_poses": eq}), flush=True)


if __name__ == "__main__":
    main()
