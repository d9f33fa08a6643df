#!/usr/bin/env python3
"""Cost of torch.cuda.synchronize() (hipDeviceSynchronize) on an idle device, and right after
a kernel, as the process gains streams: torch alone, + the engine (libdcol's side streams),
+ one torch side stream (torch then creates its stream pool), + the drop-in path's streams.
Median host microseconds of 200 calls each.

  python3 tools/sync_cost.py
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [ROOT, os.path.join(ROOT, "dcol-trajectory-optimization_amd")]


def main():
    os.environ["GPU_MAX_HW_QUEUES"] = "8"   # as bench.py
    import torch
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    x = torch.zeros(1 << 20, device=dev)

    def cost(label):
        idle, busy, one = [], [], []
        s = torch.cuda.current_stream(dev)
        for _ in range(200):
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            torch.cuda.synchronize(dev)
            idle.append((time.perf_counter() - t0) * 1e6)
        for _ in range(200):
            x.add_(1.0)
            e = torch.cuda.Event()
            e.record(s)
            while not e.query():
                pass
            t0 = time.perf_counter()
            torch.cuda.synchronize(dev)
            busy.append((time.perf_counter() - t0) * 1e6)
        for _ in range(200):
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            s.synchronize()
            one.append((time.perf_counter() - t0) * 1e6)
        print(json.dumps({"state": label, "device_sync_idle_us": float(np.median(idle)),
                          "device_sync_after_kernel_us": float(np.median(busy)),
                          "stream_sync_idle_us": float(np.median(one))}), flush=True)

    cost("torch only")
    import bench
    from dcol_amd import Engine, spec_from_arrays
    tab = bench.shape_table()
    eng = Engine(device=0)
    ids = np.array([eng.register(spec_from_arrays(tab, k)) for k in range(len(tab["type"]))], np.int32)
    cost("+ engine (side streams)")
    st = torch.cuda.Stream(dev)
    cost("+ one torch side stream (pool)")
    from primitives.misc_primitive_constructor import SphereMRP, create_rect_prism
    box = create_rect_prism(1.0, 2.0, 0.5)
    ball = SphereMRP(0.4)
    box.r, box.p = np.zeros(3), np.array([0.1, -0.2, 0.3])
    ball.r, ball.p = np.array([2.0, 0.5, -0.3]), np.zeros(3)
    eng.solve_pair(ball, box, grad=None)
    cost("+ drop-in (pair / server streams)")
    del st, ids


if __name__ == "__main__":
    main()
