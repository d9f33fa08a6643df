#!/usr/bin/env python3
"""Would splitting off the headline batch's last partial round help?  The 100k batch is
3,125 waves of the three-wave BOX kernel over 3,072 slots: the last 1,696 pairs (53 waves)
start only when the first waves end (DESIGN.md §3, 98,304 pairs 39.0 µs vs 100,000 45.3 µs).
This probe times, back to back on one stream (HIP events around each step, median of R):
  one   : the 100k plan (one BOX launch)
  split : a 98,304-pair plan (BOX) on the main stream + the last 1,696 pairs as their own
          plan on a second stream (a small plan: its latency configuration, the dense FULL
          kernel at 4 lanes per pair, 16 pairs per wave), forked / joined through events
  main  : the 98,304-pair plan alone (the floor)
Usage: python3 tools/tail_split_probe.py [R]"""
import json
import os
import statistics
import sys

import numpy as np

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."),
                os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dcol-trajectory-optimization_amd")]
import torch  # noqa: E402

torch.zeros(1, device="cuda:0")
import bench  # noqa: E402
from dcol_amd import Engine, alloc_outputs, spec_from_arrays  # noqa: E402

R = int(sys.argv[1]) if len(sys.argv) > 1 else 200
dev = torch.device("cuda", 0)
tab = bench.shape_table()
B, M = 100_000, 98_304
s1, s2, p1, p2 = bench.pairs(B, len(tab["type"]), seed=1000)
eng = Engine(device=0)
ids = np.array([eng.register(spec_from_arrays(tab, k)) for k in range(len(tab["type"]))], np.int32)
main_s = torch.cuda.current_stream(dev)
side_s = torch.cuda.Stream(dev)


def bound(lo, hi, stream):
    plan = eng.plan(ids[s1[lo:hi]], ids[s2[lo:hi]], cache=False)
    d1 = torch.from_numpy(np.ascontiguousarray(p1[lo:hi].T)).to(dev)
    d2 = torch.from_numpy(np.ascontiguousarray(p2[lo:hi].T)).to(dev)
    out = alloc_outputs(hi - lo, dev, want_grad=True, want_contact=False)
    return plan, out, plan.bind(d1, d2, out, grad="fd", contact=False, stream=stream)


p_one, o_one, one = bound(0, B, main_s)
p_main, o_main, main = bound(0, M, main_s)
p_tail, o_tail, tail = bound(M, B, side_s)
fork, join = torch.cuda.Event(), torch.cuda.Event()


def split():
    main()
    fork.record(main_s)          # (the tail's poses are already resident: the fork only orders)
    side_s.wait_event(fork)
    tail()
    join.record(side_s)
    main_s.wait_event(join)


def split_first():
    fork.record(main_s)
    side_s.wait_event(fork)
    main()
    tail()
    join.record(side_s)
    main_s.wait_event(join)


for f in (one, main, split, split_first):
    for _ in range(300):
        f()
torch.cuda.synchronize()
res = {k: [] for k in ("one", "split", "split_first", "main")}
for _ in range(R):
    for name, f in (("one", one), ("split", split), ("split_first", split_first), ("main", main)):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(main_s)
        for _ in range(10):
            f()
        b.record(main_s)
        torch.cuda.synchronize()
        res[name].append(a.elapsed_time(b) / 10 * 1e3)
torch.cuda.synchronize()
ok = bool(torch.equal(o_one["alpha"][:M], o_main["alpha"]))
st = torch.cat([o_main["status"], o_tail["status"]]).cpu().numpy()
it = torch.cat([o_main["iters"], o_tail["iters"]]).cpu().numpy()
same_iters = bool(np.array_equal(it, o_one["iters"].cpu().numpy()))
da = float((torch.cat([o_main["alpha"], o_tail["alpha"]]) - o_one["alpha"]).abs().max())
print(json.dumps({"R": R, "us_per_step_median": {k: statistics.median(v) for k, v in res.items()},
                  "us_per_step_min": {k: min(v) for k, v in res.items()},
                  "tail_buckets": p_tail.buckets(), "main_bitwise_equal_to_one": ok,
                  "iters_equal": same_iters, "all_ok": bool((st == 0).all()), "max_abs_alpha_diff": da}))
