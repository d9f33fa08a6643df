#!/usr/bin/env python3
"""Suspend / resume A/B on the benchmark batch (BASELINE configs[3], bench.py workload):
the same 100k polytope pairs through a DCOL_PLAN_SUSPEND plan and a plain plan --
bitwise comparison of every output, pairs suspended, and per-step time (HIP events, one
stream: serial; two plans on two streams: pipelined).  DCOL_SUSPEND_T / DCOL_SUSPEND_MIN set
the rule (read once per process: run one configuration per process).
Usage: DCOL_SUSPEND_T=4 DCOL_SUSPEND_MIN=6 python3 tools/susp_bench.py [--pairs 100000] [--steps 200]
"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [REPO, os.path.join(REPO, "dcol-trajectory-optimization_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=100_000)
    ap.add_argument("--steps", type=int, default=200)
    args = ap.parse_args()
    import torch

    import bench
    from dcol_amd import Engine, alloc_outputs, spec_from_arrays
    dev = torch.device("cuda", 0)
    tab = bench.shape_table()
    B = args.pairs
    s1, s2, p1, p2 = bench.pairs(B, len(tab["type"]), seed=1000)
    eng = Engine(device=0)
    ids = np.array([eng.register(spec_from_arrays(tab, k)) for k in range(len(tab["type"]))], np.int32)
    d1 = torch.from_numpy(np.ascontiguousarray(p1.T)).to(dev)
    d2 = torch.from_numpy(np.ascontiguousarray(p2.T)).to(dev)
    streams = [torch.cuda.current_stream(dev), torch.cuda.Stream(dev)]
    res = {"T": os.environ.get("DCOL_SUSPEND_T", "4"), "min": os.environ.get("DCOL_SUSPEND_MIN", "6"), "pairs": B}
    outs = {}
    for name, susp in (("plain", False), ("suspend", True)):
        plans = [eng.plan(ids[s1], ids[s2], cache=False, suspend=susp) for _ in streams]
        os_ = [alloc_outputs(B, dev, True, False) for _ in streams]
        runs = [pl.bind(d1, d2, o, grad="fd", contact=False, stream=st) for pl, o, st in zip(plans, os_, streams)]
        for _ in range(50):
            runs[0]()
        torch.cuda.synchronize(dev)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
        for e0, e1 in ev:
            e0.record(streams[0])
            runs[0]()
            e1.record(streams[0])
        torch.cuda.synchronize(dev)
        serial = float(np.median([a.elapsed_time(b) for a, b in ev]))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(dev)
        e0.record(streams[0])
        for k in range(args.steps):
            runs[k % 2]()
        for st in streams[1:]:
            streams[0].wait_stream(st)
        e1.record(streams[0])
        torch.cuda.synchronize(dev)
        piped = e0.elapsed_time(e1) / args.steps
        runs[0]()
        torch.cuda.synchronize(dev)
        outs[name] = {k: v.cpu().numpy() for k, v in os_[0].items()}
        res[name] = {"serial_ms": serial, "pipelined_ms_per_step": piped, "pipelined_pairs_per_s": B / (piped * 1e-3),
                     "suspended": plans[0].suspended() if susp else 0,
                     "launches": plans[0].num_launches}
    a, b = outs["plain"], outs["suspend"]
    res["bitwise_equal"] = {k: bool(np.array_equal(a[k], b[k], equal_nan=True)) for k in a}
    res["iters_mean"] = float(a["iters"].mean())
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
