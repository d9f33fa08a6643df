#!/usr/bin/env python3
"""Host-side cost of issuing a plan (round-3 mixed1m investigation).

Builds the configs[4] plan (1M mixed pairs, ~16 variant launches) and the configs[3] plan
(100k polytope pairs, one launch), then for each: the host time of K back-to-back
asynchronous dcol_plan_run calls (no synchronisation in between) and the GPU time of the
same K runs (HIP events on the launch stream).  host_ms_per_run >= gpu_ms_per_run means the
run is bound by issuing, not by the kernels.  Usage: python3 tools/launch_probe.py [K]
(set DCOL_NO_FANOUT=1 for the one-stream plan)."""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "dcol-trajectory-optimization_amd")]


def probe(name, tab, s1, s2, p1, p2, K):
    import torch
    from dcol_amd import Engine, alloc_outputs, spec_from_arrays
    eng = Engine(device=0)
    ids = np.array([eng.register(spec_from_arrays(tab, k)) for k in range(len(tab["type"]))], np.int32)
    plan = eng.plan(ids[s1], ids[s2])
    d1 = torch.from_numpy(np.ascontiguousarray(p1.T)).cuda()
    d2 = torch.from_numpy(np.ascontiguousarray(p2.T)).cuda()
    out = alloc_outputs(len(s1), "cuda", want_grad=True, want_contact=False)
    st = torch.cuda.current_stream()
    launch = plan.bind(d1, d2, out, grad="fd", contact=False, stream=st)
    for _ in range(3):
        launch()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    t0 = time.perf_counter()
    for _ in range(K):
        launch()
    host = time.perf_counter() - t0
    e1.record(st)
    torch.cuda.synchronize()
    gpu = e0.elapsed_time(e1) / K
    # GPU time of one run issued alone (the queue drained before and after)
    one = []
    for _ in range(5):
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        launch()
        b.record(st)
        torch.cuda.synchronize()
        one.append(a.elapsed_time(b))
    print(f"{name:10s} launches {plan.num_launches:3d}  host_ms_per_run {1e3 * host / K:7.3f}  "
          f"gpu_ms_per_run(back-to-back) {gpu:7.3f}  gpu_ms_one_run {np.median(one):7.3f}  "
          f"host_us_per_launch {1e6 * host / K / plan.num_launches:6.1f}", flush=True)


def main():
    import bench
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    tab = bench.mixed_table()
    s1, s2, p1, p2 = bench.mixed_pairs(tab, 1_000_000, seed=0)
    probe("mixed1m", tab, s1, s2, p1, p2, K)
    tab = bench.shape_table()
    s1, s2, p1, p2 = bench.pairs(100_000, len(tab["type"]), seed=1000)
    probe("poly100k", tab, s1, s2, p1, p2, K)


if __name__ == "__main__":
    main()
