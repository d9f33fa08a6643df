#!/usr/bin/env python3
"""Two 1M-pair poly x poly batches of the same distribution (bench.py pairs(), seeds 7 and
1000), one launch each, alternated in one process after a common warm-up: per-launch HIP-event
time, mean / per-wave-max Newton iterations.  Does the batch itself, not the clock state, set
kernel_1m's 0.425 ms against the 0.365 ms of `bench.py --pairs 1000000`?
Usage: python3 tools/seed_probe.py"""
import json
import os
import sys

import numpy as np

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [REPO, os.path.join(REPO, "dcol-trajectory-optimization_amd")]


def main():
    import torch

    import bench
    from dcol_amd import Engine, alloc_outputs, spec_from_arrays
    dev = torch.device("cuda", 0)
    eng = Engine(device=0)
    tab = bench.shape_table()
    ids = np.array([eng.register(spec_from_arrays(tab, k)) for k in range(len(tab["type"]))], np.int32)
    B = 1_000_000
    stream = torch.cuda.current_stream(dev)
    runs = {}
    for seed in (7, 1000):
        s1, s2, p1, p2 = bench.pairs(B, len(tab["type"]), seed=seed)
        plan = eng.plan(ids[s1], ids[s2], cache=False)
        d1 = torch.from_numpy(np.ascontiguousarray(p1.T)).to(dev)
        d2 = torch.from_numpy(np.ascontiguousarray(p2.T)).to(dev)
        out = alloc_outputs(B, dev, want_grad=True, want_contact=False)
        runs[seed] = (plan.bind(d1, d2, out, grad="fd", contact=False, stream=stream), out, plan, d1, d2)
    for _ in range(20):
        for seed in runs:
            runs[seed][0]()
    ev = {seed: [] for seed in runs}
    for _ in range(20):
        for seed in runs:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            runs[seed][0]()
            e1.record(stream)
            ev[seed].append((e0, e1))
    torch.cuda.synchronize(dev)
    for seed in runs:
        it = runs[seed][1]["iters"].cpu().numpy()
        waves = it[: (B // 32) * 32].reshape(-1, 32).max(axis=1)
        print(json.dumps({"seed": seed, "ms_median": float(np.median([a.elapsed_time(b) for a, b in ev[seed]])),
                          "iters_mean": float(it.mean()), "wave_max_mean": float(waves.mean())}), flush=True)


if __name__ == "__main__":
    main()
