#!/usr/bin/env python3
"""Print the variant buckets of the 1M mixed plan (bench.py --workload mixed1m, configs[4]):
key, pairs, lanes per pair, the host's cost estimate (dcol_capi.cpp bucket_cost) -- to pair
with a rocprofv3 kernel trace of the same plan (tools/session_r05r.sh)."""
import json
import os
import sys

import numpy as np

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."),
                os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dcol-trajectory-optimization_amd")]
import bench  # noqa: E402
from dcol_amd import Engine, spec_from_arrays  # noqa: E402


def cost(b):
    dense_soc = b["nsoc"] > 0 and not (b["flags"] & 6)
    per = 0.0806 * b["omax"] + 0.127 * b["nsoc"] + 0.0139 * b["N"] ** 2 + (0.143 * b["nsoc"] if dense_soc else 0.0)
    return b["pairs"] * per * (0.5 if b["nsoc"] == 0 else 1.0)


if "--steps" in sys.argv:   # torch's HIP context first (as bench.py does), then the engine's
    import torch
    torch.zeros(1, device="cuda:0")
tab = bench.mixed_table()
s1, s2, _, _ = bench.mixed_pairs(tab, 1_000_000, seed=0)
eng = Engine(device=0)
ids = np.array([eng.register(spec_from_arrays(tab, k)) for k in range(len(tab["type"]))], np.int32)
plan = eng.plan(ids[s1], ids[s2], cache=False)
for b in plan.buckets():
    b["cost_est_us"] = round(cost(b) / 1e3, 1)
    print(json.dumps(b))

# --steps K: K solves of the plan one at a time (synchronised between steps, so a kernel
# trace of this process separates the steps cleanly), with the step's wall time by HIP events
if "--steps" in sys.argv:
    import torch
    K = int(sys.argv[sys.argv.index("--steps") + 1])
    _, _, p1, p2 = bench.mixed_pairs(tab, 1_000_000, seed=0)
    dev = torch.device("cuda", 0)
    d1 = torch.from_numpy(np.ascontiguousarray(p1.T)).to(dev)
    d2 = torch.from_numpy(np.ascontiguousarray(p2.T)).to(dev)
    from dcol_amd import alloc_outputs
    out = alloc_outputs(plan.B, dev, want_grad=True, want_contact=False)
    for _ in range(10):
        plan.run(d1, d2, grad="fd", contact=False, out=out)
    torch.cuda.synchronize()
    ms = []
    for _ in range(K):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        plan.run(d1, d2, grad="fd", contact=False, out=out)
        b.record()
        torch.cuda.synchronize()
        ms.append(a.elapsed_time(b))
    print(json.dumps({"steps": K, "step_ms_median": float(np.median(ms)), "step_ms_min": float(np.min(ms)),
                      "fanout": os.environ.get("DCOL_NO_FANOUT") is None}))
