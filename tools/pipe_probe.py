#!/usr/bin/env python3
"""bench.py's pipelined issue (configs[3]: K steps round-robin on S streams, each stream with
its own outputs) as a function of K and S, beside the one-stream rate: is the overlap rate a
property of the queue depth?  Prints one JSON line per (S, K): host wall ms per step (polling
the last events), and the number of launches the host had issued when the first step
finished (the queue depth the run reached).

  python3 tools/pipe_probe.py [--ks 20,50,100,200,500] [--streams 1,2,3]
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
    ap.add_argument("--ks", default="20,50,100,200,500")
    ap.add_argument("--streams", default="1,2,3")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--hw-queues", default="8", help="GPU_MAX_HW_QUEUES (bench.py's default)")
    a = ap.parse_args()
    os.environ.setdefault("GPU_MAX_HW_QUEUES", a.hw_queues)
    import torch

    import bench
    from dcol_amd import Engine, alloc_outputs, spec_from_arrays
    dev = torch.device("cuda", 0)
    torch.zeros(1, device=dev)
    tab = bench.shape_table()
    B = 100_000
    s1, s2, p1, p2 = bench.pairs(B, len(tab["type"]), seed=1000)
    eng = Engine(device=0)
    ids = np.array([eng.register(spec_from_arrays(tab, k)) for k in range(len(tab["type"]))], np.int32)
    plan = eng.plan(ids[s1], ids[s2])
    d1 = torch.from_numpy(np.ascontiguousarray(p1.T)).to(dev)
    d2 = torch.from_numpy(np.ascontiguousarray(p2.T)).to(dev)
    smax = max(int(x) for x in a.streams.split(","))
    streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(smax - 1)]
    lanes = [plan.bind(d1, d2, alloc_outputs(B, dev, want_grad=True, want_contact=False), grad="fd", contact=False,
                       stream=st) for st in streams]
    bench.clock_settle(lanes[0], streams[0], dev, None, 30.0)
    for S in [int(x) for x in a.streams.split(",")]:
        for K in [int(x) for x in a.ks.split(",")]:
            ms, depth = [], []
            for _ in range(a.reps):
                for k in range(20):
                    lanes[k % S]()
                torch.cuda.synchronize(dev)
                done = []
                t0 = time.perf_counter()
                first_seen = None
                for k in range(K):
                    lanes[k % S]()
                    e = torch.cuda.Event()
                    e.record(streams[k % S])
                    done.append(e)
                    if first_seen is None and done[0].query():
                        first_seen = k + 1
                for e in done:
                    while not e.query():
                        pass
                torch.cuda.synchronize(dev)
                ms.append((time.perf_counter() - t0) * 1e3 / K)
                depth.append(first_seen or K)
            print(json.dumps({"streams": S, "steps": K, "ms_per_step": float(np.median(ms)),
                              "pair_solves_per_s": B / (float(np.median(ms)) * 1e-3),
                              "issued_when_first_done": int(np.median(depth))}), flush=True)


if __name__ == "__main__":
    main()
