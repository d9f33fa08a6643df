#!/usr/bin/env python3
"""Where the driver-length line's ms_per_step exceeds its kernel_ms: the host-side cost of
the timed region's bracket (K = 20 steps of the 100k plan, bench.py's headline).  Each
variant repeats the bracket R times and reports median wall / K, event / K and their
difference ("overhead per step"); interleaved.
  A  bench.py's bracket: sync, t0, event, K steps, event, event.synchronize(), sync, t1
  B  the same, the end event polled with query() in a spin loop before the synchronize
  C  B without the start event (the region's first launch issued straight after t0)
  D  an empty bracket (no steps): sync, t0, event, event, synchronize, sync, t1 -- the floor
EXTRA_STREAM=1 creates one torch side stream first (bench.py's pipeline lane); run it with
GPU_MAX_HW_QUEUES=8 as bench.py does (--hw-queues).
"""
import json
import os
import statistics
import sys
import time

import numpy as np

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."),
                os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dcol-trajectory-optimization_amd")]
import torch  # noqa: E402

torch.zeros(1, device="cuda:0")
import bench  # noqa: E402
from dcol_amd import Engine, alloc_outputs, spec_from_arrays  # noqa: E402

K = int(os.environ.get("K", "20"))
R = int(os.environ.get("R", "15"))
dev = torch.device("cuda", 0)
tab = bench.shape_table()
B = 100_000
s1, s2, p1, p2 = bench.pairs(B, len(tab["type"]), seed=1000)
eng = Engine(device=0)
ids = np.array([eng.register(spec_from_arrays(tab, k)) for k in range(len(tab["type"]))], np.int32)
plan = eng.plan(ids[s1], ids[s2])
pose1 = torch.from_numpy(np.ascontiguousarray(p1.T)).to(dev)
pose2 = torch.from_numpy(np.ascontiguousarray(p2.T)).to(dev)
out = alloc_outputs(B, dev, want_grad=True, want_contact=False)
stream = torch.cuda.current_stream(dev)
if os.environ.get("EXTRA_STREAM"):   # as bench.py's pipeline lane (torch then creates its stream pool)
    extra = torch.cuda.Stream(dev)
step = plan.bind(pose1, pose2, out, grad="fd", contact=False, stream=stream)
for _ in range(600):
    step()
torch.cuda.synchronize(dev)


def bracket(kind):
    torch.cuda.synchronize(dev)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    if kind != "C":
        a.record(stream)
    for _ in range(K if kind != "D" else 0):
        step()
        if kind == "C" and _ == 0:
            pass
    b.record(stream)
    if kind in ("B", "C"):
        while not b.query():
            pass
    b.synchronize()
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    ev = a.elapsed_time(b) / 1e3 if kind != "C" else float("nan")
    return wall, ev


res = {k: [] for k in "ABCD"}
for r in range(R):
    for k in "ABCD":
        res[k].append(bracket(k))
out_ = {}
for k, v in res.items():
    w = statistics.median(x[0] for x in v)
    e = statistics.median(x[1] for x in v) if k not in "C" else float("nan")
    n = K if k != "D" else 1
    out_[k] = {"wall_us_per_step": 1e6 * w / n, "event_us_per_step": 1e6 * e / n,
               "overhead_us_total": 1e6 * (w - e) if k not in "C" else None}
print(json.dumps({"K": K, "R": R, **out_}))
