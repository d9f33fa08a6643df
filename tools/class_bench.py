#!/usr/bin/env python3
"""Per-pair-class throughput of the solve kernels (one class per plan, one launch at a
time, HIP events): which kernel variants the mixed workload (bench.py --workload mixed1m)
and the scene batches spend their time in.

For every ordered kind pair of the mixed workload (27 supported ones), B pairs of only that
class are solved with FD gradients; prints per class the variant launched, pair-solves/s,
kernel ms and mean / max Newton iterations.  Also times a latency-size batch (default 1,000
pairs) per class.
Each class line also carries its FP64 roofline fraction: the reference's COUNTED flops per
pair (profiles/flop_model.json, oracle/dcol_oracle_opcount.cpp: assembly + pdip_fixed +
pdip_per_iter x the batch's measured mean iterations + FD gradient) x pairs / kernel time,
against the 78.6 TF/s FP64 vector peak (MI355X_MICROARCH.md).
Usage: python3 tools/class_bench.py [--pairs 200000] [--small 1000 (0: skip)] [--reps 10] [--classes a-b,...]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "dcol-trajectory-optimization_amd"))

import bench  # noqa: E402

FP64_PEAK = 78.6e12
NAMES = {0: "polytope", 1: "sphere", 2: "cone", 3: "capsule", 4: "cylinder", 5: "polygon"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=200_000)
    ap.add_argument("--small", type=int, default=1000)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--classes", default="", help="comma-separated class names (default: all 27)")
    args = ap.parse_args()
    import torch
    from dcol_amd import Engine, alloc_outputs, spec_from_arrays
    dev = torch.device("cuda", 0)
    tab = bench.mixed_table()
    eng = Engine(device=0)
    ids = np.array([eng.register(spec_from_arrays(tab, k)) for k in range(len(tab["type"]))], np.int32)
    by_kind = {k: np.flatnonzero(tab["type"] == k) for k in bench.MIXED_KINDS}
    combos = [(a, b) for a in bench.MIXED_KINDS for b in bench.MIXED_KINDS if a <= 2 or b <= 2]
    fm = json.load(open(os.path.join(REPO, "profiles", "flop_model.json")))["classes"]
    rng = np.random.default_rng(0)
    stream = torch.cuda.current_stream(dev)
    rows = []
    if args.classes:
        want = set(args.classes.split(","))
        combos = [(a, b) for a, b in combos if f"{NAMES[a]}-{NAMES[b]}" in want]
    for a, b in combos:
        rec = {"class": f"{NAMES[a]}-{NAMES[b]}"}
        for label, B in (("big", args.pairs), ("small", args.small)):
            if B <= 0:
                continue
            s1 = rng.choice(by_kind[a], B).astype(np.int32)
            s2 = rng.choice(by_kind[b], B).astype(np.int32)
            p1 = np.hstack([rng.uniform(-3, 3, (B, 3)), rng.uniform(-1, 1, (B, 3))])
            p2 = np.hstack([rng.uniform(-3, 3, (B, 3)), rng.uniform(-1, 1, (B, 3))])
            plan = eng.plan(ids[s1], ids[s2], cache=False)
            d1 = torch.from_numpy(np.ascontiguousarray(p1.T)).to(dev)
            d2 = torch.from_numpy(np.ascontiguousarray(p2.T)).to(dev)
            out = alloc_outputs(B, dev, want_grad=True, want_contact=False)
            run = plan.bind(d1, d2, out, grad="fd", contact=False, stream=stream)
            run()
            torch.cuda.synchronize(dev)
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.reps)]
            for e0, e1 in ev:
                e0.record(stream)
                run()
                e1.record(stream)
            torch.cuda.synchronize(dev)
            ms = float(np.median([x.elapsed_time(y) for x, y in ev]))
            it = out["iters"].cpu().numpy()
            st = out["status"].cpu().numpy()
            rec[label] = {"pairs": B, "kernel_ms": round(ms, 4), "pair_solves_per_s": B / (ms * 1e-3),
                          "iters_mean": round(float(it[st == 0].mean()), 2), "iters_max": int(it.max()),
                          "ok_frac": float(np.mean(st == 0)), "launches": plan.num_launches}
            m = fm.get(rec["class"])
            if m:   # counted flops at this batch's mean iteration count
                fl = m["assembly"] + m["pdip_fixed"] + m["pdip_per_iter"] * float(it[st == 0].mean()) + m["grad_fd"]
                rec[label]["flops_per_pair"] = round(fl, 1)
                rec[label]["fp64_roofline_frac"] = round(fl * B / (ms * 1e-3) / FP64_PEAK, 4)
        rows.append(rec)
        print(json.dumps(rec), flush=True)
    tot_big = sum(r["big"]["pairs"] / r["big"]["pair_solves_per_s"] for r in rows)
    print(json.dumps({"harmonic_mix_pair_solves_per_s": len(rows) * args.pairs / tot_big}), flush=True)


if __name__ == "__main__":
    main()
