#!/usr/bin/env python3
"""Where the fixed cost of bench.py's timed region goes (configs[3], K = 20 as the driver
runs it): the region is repeated exactly as bench.py times it (synchronize, t0, event, K
steps, event, poll, synchronize) after the same settle + warm-up, and each repetition prints
its host wall time, its event span, and -- in the probe variants -- the host time until the
first step() returned and until the start event had executed.

  python3 tools/region_probe.py [--steps 20] [--reps 8]
Variants (one line each per repetition):
  bench     bench.py's sequence
  idle1ms   the same after 1 ms of host sleep (GPU idle) before t0
  startpoll the start event polled to completion before the first step (its dispatch latency
            measured on its own; the steps then start from a busy-polled queue)
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
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--reps", type=int, default=8)
    a = ap.parse_args()
    os.environ["GPU_MAX_HW_QUEUES"] = "8"   # as bench.py
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
    out = alloc_outputs(B, dev, want_grad=True, want_contact=False)
    stream = torch.cuda.current_stream(dev)
    step = plan.bind(d1, d2, out, grad="fd", contact=False, stream=stream)
    bench.clock_settle(step, stream, dev, None, 30.0)
    for _ in range(5):
        step()
    torch.cuda.synchronize(dev)
    K = a.steps
    for rep in range(a.reps):
        for variant in ("bench", "idle1ms", "startpoll"):
            torch.cuda.synchronize(dev)
            if variant == "idle1ms":
                time.sleep(0.001)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0 = time.perf_counter()
            e0.record(stream)
            t_start = None
            if variant == "startpoll":
                while not e0.query():
                    pass
                t_start = time.perf_counter()
            step()
            t_first = time.perf_counter()
            for _ in range(K - 1):
                step()
            t_issued = time.perf_counter()
            e1.record(stream)
            while not e1.query():
                pass
            t_done = time.perf_counter()
            torch.cuda.synchronize(dev)
            t1 = time.perf_counter()
            ev = e0.elapsed_time(e1)
            r = {"rep": rep, "variant": variant, "wall_ms": (t1 - t0) * 1e3, "event_ms": ev,
                 "fixed_ms": (t1 - t0) * 1e3 - ev, "first_step_return_ms": (t_first - t0) * 1e3,
                 "all_issued_ms": (t_issued - t0) * 1e3, "seen_done_ms": (t_done - t0) * 1e3}
            if t_start is not None:
                r["start_event_done_ms"] = (t_start - t0) * 1e3
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
