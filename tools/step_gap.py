#!/usr/bin/env python3
"""Where the serial step's time goes beyond the kernel: K back-to-back launches of the 100k
poly x poly plan on one stream (a) plain, (b) with HIP events around every launch, (c) as
one captured hipGraph of K launches, (d) the same graph with event nodes around every
launch.  Prints ms per step and, where events exist, the mean kernel interval.
Usage: python3 tools/step_gap.py [--steps 20] [--reps 5]"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(REPO, "dcol-trajectory-optimization_amd"), REPO]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import torch
    import bench
    from dcol_amd import Engine, alloc_outputs, spec_from_arrays
    dev = torch.device("cuda", 0)
    tab = bench.shape_table()
    s1, s2, p1, p2 = bench.pairs(100_000, 64, seed=1000)
    eng = Engine(device=0)
    ids = np.array([eng.register(spec_from_arrays(tab, k)) for k in range(64)], np.int32)
    plan = eng.plan(ids[s1], ids[s2])
    d1 = torch.from_numpy(np.ascontiguousarray(p1.T)).to(dev)
    d2 = torch.from_numpy(np.ascontiguousarray(p2.T)).to(dev)
    out = alloc_outputs(100_000, dev, want_grad=True, want_contact=False)
    st = torch.cuda.Stream(dev)
    step = plan.bind(d1, d2, out, grad="fd", contact=False, stream=st)
    K = a.steps
    bench.clock_settle(step, st, dev, None, 30.0)

    def ev():
        return torch.cuda.Event(enable_timing=True)

    def plain():
        for _ in range(K):
            step()

    evs = [(ev(), ev()) for _ in range(K)]

    def with_events():
        for e0, e1 in evs:
            e0.record(st)
            step()
            e1.record(st)

    g_plain = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g_plain, stream=st):
        plain()
    gevs = [(ev(), ev()) for _ in range(K)]
    g_ev = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g_ev, stream=st):
        for e0, e1 in gevs:
            e0.record(st)
            step()
            e1.record(st)
    res = {}
    for name, fn, pairs_ in (("plain", plain, None), ("events", with_events, evs),
                             ("graph", g_plain.replay, None), ("graph_events", g_ev.replay, gevs)):
        ts, ks = [], []
        for _ in range(a.reps):
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            with torch.cuda.stream(st):
                fn()
            st.synchronize()
            ts.append(1e3 * (time.perf_counter() - t0) / K)
            if pairs_ is not None:
                try:
                    ks.append(float(np.mean([x.elapsed_time(y) for x, y in pairs_])))
                except Exception as e:   # timing events inside a graph may be unsupported
                    ks.append(repr(e)[:80])
        res[name] = {"ms_per_step": float(np.median(ts)), "all": ts, "kernel_ms": ks or None}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
