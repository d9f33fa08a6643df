#!/usr/bin/env python3
"""configs[3]'s timed region as plain launches against one HIP graph of the same K steps
(torch.cuda.CUDAGraph capture of K plan runs on a side stream, replayed on it): host wall time
of the region (synchronize, t0, K steps / one replay, polled end event, synchronize) and the
event span, per K, median of --reps regions.  Also checks the graph's outputs bitwise against
the plain launches'.

  python3 tools/graph_probe.py [--ks 1,5,20,100] [--reps 9]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [ROOT, os.path.join(ROOT, "dcol-trajectory-optimization_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ks", default="1,5,20,100")
    ap.add_argument("--reps", type=int, default=9)
    a = ap.parse_args()
    os.environ["GPU_MAX_HW_QUEUES"] = "8"
    import torch

    import bench
    from dcol_amd import Engine, alloc_outputs, spec_from_arrays
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    tab = bench.shape_table()
    B = 100_000
    s1, s2, p1, p2 = bench.pairs(B, len(tab["type"]), seed=1000)
    eng = Engine(device=0)
    ids = np.array([eng.register(spec_from_arrays(tab, k)) for k in range(len(tab["type"]))], np.int32)
    plan = eng.plan(ids[s1], ids[s2])
    d1 = torch.from_numpy(np.ascontiguousarray(p1.T)).to(dev)
    d2 = torch.from_numpy(np.ascontiguousarray(p2.T)).to(dev)
    s = torch.cuda.Stream(dev)
    out = alloc_outputs(B, dev, want_grad=True, want_contact=False)
    step = plan.bind(d1, d2, out, grad="fd", contact=False, stream=s)
    with torch.cuda.stream(s):
        bench.clock_settle(step, s, dev, None, 30.0)
        for _ in range(20):
            step()
    torch.cuda.synchronize(dev)
    ref = {k: v.clone() for k, v in out.items()}
    graphs = {}
    for K in [int(x) for x in a.ks.split(",")]:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(K):
                step()
        graphs[K] = g
    torch.cuda.synchronize(dev)
    for K, g in graphs.items():
        for mode in ("plain", "graph", "plain", "graph"):
            walls, evs = [], []
            for _ in range(a.reps):
                torch.cuda.synchronize(dev)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                t0 = time.perf_counter()
                e0.record(s)
                if mode == "plain":
                    for _ in range(K):
                        step()
                else:
                    with torch.cuda.stream(s):
                        g.replay()
                e1.record(s)
                while not e1.query():
                    pass
                torch.cuda.synchronize(dev)
                walls.append((time.perf_counter() - t0) * 1e3)
                evs.append(e0.elapsed_time(e1))
            same = all(torch.equal(out[k].view(torch.int64) if out[k].dtype == torch.float64 else out[k],
                                   ref[k].view(torch.int64) if ref[k].dtype == torch.float64 else ref[k]) for k in out)
            print(json.dumps({"K": K, "mode": mode, "wall_ms_per_step": float(np.median(walls)) / K,
                              "event_ms_per_step": float(np.median(evs)) / K,
                              "fixed_ms": float(np.median(walls)) - float(np.median(evs)),
                              "bitwise_equal": same}), flush=True)


if __name__ == "__main__":
    main()
