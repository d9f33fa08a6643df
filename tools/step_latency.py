#!/usr/bin/env python3
"""Fixed overhead of bench.py's timed region (configs[3], one stream): host wall time of K
back-to-back steps bracketed by synchronize, for several K, ended either by
torch.cuda.synchronize() alone or by spinning on the last step's event first (then the same
synchronize).  The intercept of wall time over K is the region's fixed cost (first dispatch
from an idle queue + the host's wake-up at the end); the slope is the per-step time.

  python3 tools/step_latency.py [--ks 1,2,5,10,20,50] [--reps 7]
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
    ap.add_argument("--ks", default="1,2,5,10,20,50")
    ap.add_argument("--reps", type=int, default=7)
    a = ap.parse_args()
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
    out = alloc_outputs(B, dev, want_grad=True, want_contact=False)
    stream = torch.cuda.current_stream(dev)
    step = plan.bind(d1, d2, out, grad="fd", contact=False, stream=stream)
    bench.clock_settle(step, stream, dev, None, 30.0)
    for _ in range(50):
        step()
    torch.cuda.synchronize(dev)
    ks = [int(x) for x in a.ks.split(",")]
    res = {}
    for mode in ("sync", "spin", "sync", "spin"):
        for K in ks:
            ts, ev = [], []
            for _ in range(a.reps):
                torch.cuda.synchronize(dev)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                t0 = time.perf_counter()
                e0.record(stream)
                for _ in range(K):
                    step()
                e1.record(stream)
                if mode == "spin":
                    while not e1.query():
                        pass
                torch.cuda.synchronize(dev)
                ts.append((time.perf_counter() - t0) * 1e3)
                ev.append(e0.elapsed_time(e1))
            res.setdefault(mode, {}).setdefault(K, []).append((float(np.median(ts)), float(np.median(ev))))
    for mode, byk in res.items():
        xs = np.array(ks, float)
        wall = np.array([np.median([w for w, _ in byk[k]]) for k in ks])
        evt = np.array([np.median([e for _, e in byk[k]]) for k in ks])
        sl, ic = np.polyfit(xs, wall, 1)
        esl, eic = np.polyfit(xs, evt, 1)
        print(json.dumps({"end": mode, "wall_ms": dict(zip(ks, wall.round(4).tolist())),
                          "event_ms": dict(zip(ks, evt.round(4).tolist())),
                          "wall_fit": {"ms_per_step": sl, "fixed_ms": ic},
                          "event_fit": {"ms_per_step": esl, "fixed_ms": eic}}), flush=True)
    # the first dispatch alone: an empty torch kernel from an idle queue, host wall to completion
    ts = []
    for _ in range(20):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        torch.cuda._sleep(1)
        torch.cuda.synchronize(dev)
        ts.append((time.perf_counter() - t0) * 1e3)
    print(json.dumps({"tiny_kernel_roundtrip_ms": float(np.median(ts))}), flush=True)


if __name__ == "__main__":
    main()
