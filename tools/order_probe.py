#!/usr/bin/env python3
"""Slot order of configs[3]'s 100k poly x poly plan against the kernel time.  A wave of 32
pairs runs until its slowest pair has converged (iterations 5-15, mean 7.0), so the order in
which pairs fill waves matters: pairs of similar iteration count in one wave waste fewer
lane-iterations.  Orders: as given (random), sorted by the iteration counts of a previous
solve (descending / ascending), and -- the realistic case -- sorted by the counts of a
solve at slightly different poses (a trajectory optimiser's previous iterate: r + N(0, sr),
p + N(0, sp)) and timed at the new poses.  Every order's outputs are checked bitwise against
the given order's (a pair's arithmetic does not depend on its slot).

  python3 tools/order_probe.py [--reps 200] [--sr 0.01] [--sp 0.005]
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
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--sr", type=float, default=0.01)
    ap.add_argument("--sp", type=float, default=0.005)
    ap.add_argument("--pairs", type=int, default=100_000)
    a = ap.parse_args()
    import torch

    import bench
    from dcol_amd import Engine, alloc_outputs, spec_from_arrays
    dev = torch.device("cuda", 0)
    torch.zeros(1, device=dev)
    tab = bench.shape_table()
    B = a.pairs
    s1, s2, p1, p2 = bench.pairs(B, len(tab["type"]), seed=1000)
    rng = np.random.default_rng(5)
    q1, q2 = p1.copy(), p2.copy()   # the "next iterate": small pose changes
    for q in (q1, q2):
        q[:, :3] += rng.normal(0, a.sr, (B, 3))
        q[:, 3:] += rng.normal(0, a.sp, (B, 3))
    eng = Engine(device=0)
    ids = np.array([eng.register(spec_from_arrays(tab, k)) for k in range(len(tab["type"]))], np.int32)
    stream = torch.cuda.current_stream(dev)

    def run(order, P1, P2, reps):
        plan = eng.plan(ids[s1[order]], ids[s2[order]], cache=False)
        d1 = torch.from_numpy(np.ascontiguousarray(P1[order].T)).to(dev)
        d2 = torch.from_numpy(np.ascontiguousarray(P2[order].T)).to(dev)
        out = alloc_outputs(B, dev, want_grad=True, want_contact=False)
        step = plan.bind(d1, d2, out, grad="fd", contact=False, stream=stream)
        for _ in range(40):
            step()
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            step()
        e1.record(stream)
        torch.cuda.synchronize(dev)
        inv = np.empty(B, np.int64)
        inv[order] = np.arange(B)
        res = {k: out[k].cpu().numpy()[inv] if out[k].dim() == 1 else out[k].cpu().numpy()[:, inv]
               for k in ("alpha", "iters", "status", "grad")}
        return e0.elapsed_time(e1) / reps, res

    ident = np.arange(B)
    run(ident, p1, p2, 50)                       # clocks up
    t0, r0 = run(ident, p1, p2, a.reps)
    it = r0["iters"]
    desc = np.argsort(-it, kind="stable")
    asc = np.argsort(it, kind="stable")
    lines = [{"order": "given", "poses": "p", "kernel_ms": t0}]
    for name, order in (("iters_desc", desc), ("iters_asc", asc), ("random", rng.permutation(B))):
        t, r = run(order, p1, p2, a.reps)
        same = all(np.array_equal(r[k], r0[k]) for k in r0)
        lines.append({"order": name, "poses": "p", "kernel_ms": t, "bitwise_equal_to_given": same})
    # previous-iterate prediction: order from p's counts, timed at the perturbed poses q
    tq0, rq0 = run(ident, q1, q2, a.reps)
    itq = rq0["iters"]
    tq, rq = run(desc, q1, q2, a.reps)
    same = all(np.array_equal(rq[k], rq0[k]) for k in rq0)
    lines.append({"order": "given", "poses": "q", "kernel_ms": tq0})
    lines.append({"order": "iters_desc of p", "poses": "q", "kernel_ms": tq, "bitwise_equal_to_given": same,
                  "iters_changed_frac": float(np.mean(itq != it)), "iters_mean_p": float(it.mean()),
                  "iters_mean_q": float(itq.mean())})
    tqo, _ = run(np.argsort(-itq, kind="stable"), q1, q2, a.reps)
    lines.append({"order": "iters_desc of q (oracle order)", "poses": "q", "kernel_ms": tqo})
    # wave-level waste: sum over waves of 32 x max - sum of iterations
    def waste(order, its):
        w = its[order][: (B // 32) * 32].reshape(-1, 32)
        return float((w.max(1).sum() * 32 - w.sum()) / w.sum())
    print(json.dumps({"lane_iteration_waste": {"given": waste(ident, it), "iters_desc": waste(desc, it),
                                               "q_given": waste(ident, itq), "q_by_p_desc": waste(desc, itq)}}))
    for l in lines:
        print(json.dumps(l), flush=True)


if __name__ == "__main__":
    main()
