#!/usr/bin/env python3
"""Counted FP64 flop model per pair class -> profiles/flop_model.json (the
op-counter mode of the C restatement gives the official flops_per_pair).

For each class, solves a seeded sample with oracle/dcol_oracle_opcount.cpp (every +, -, *,
/, sqrt of the reference's algorithm = 1) and fits
    flops(pair) = assembly + pdip_fixed + pdip_per_iter * iters + grad_fd
(assembly and the FD gradient are per-class constants up to data-dependent branches; the
PDIP part is least-squares linear in the Newton iteration count).  bench.py evaluates the
model at the GPU run's mean iteration count.
Classes: the benchmark's poly6-poly6 (bench.shape_table / bench.pairs) and the 27 ordered
kind pairs of the mixed workload (bench.mixed_table).
Usage: python tests/golden/gen_flop_model.py [--pairs 2000]
"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, REPO)

NAMES = {0: "polytope", 1: "sphere", 2: "cone", 3: "capsule", 4: "cylinder", 5: "polygon"}


def fit(oc):
    ok = oc["status"] == 0
    it = oc["iters"][ok].astype(np.float64)
    pd = oc["pdip"][ok].astype(np.float64)
    A = np.vstack([np.ones_like(it), it]).T
    (c0, c1), *_ = np.linalg.lstsq(A, pd, rcond=None)
    tot = oc["assembly"][ok] + oc["pdip"][ok] + oc["grad"][ok]
    return {"assembly": float(oc["assembly"][ok].mean()), "pdip_fixed": float(c0), "pdip_per_iter": float(c1),
            "grad_fd": float(oc["grad"][ok].mean()), "mean_iters": float(it.mean()),
            "mean_total": float(tot.mean()), "pairs": int(ok.sum()),
            "pdip_fit_max_abs_err": float(np.abs(A @ np.array([c0, c1]) - pd).max())}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=2000)
    args = ap.parse_args()
    import bench
    from oracle import c_oracle
    model = {"units": "FP64 ops per pair (+ - * / sqrt = 1), counted by oracle/dcol_oracle_opcount.cpp",
             "formula": "assembly + pdip_fixed + pdip_per_iter * iters + grad_fd", "classes": {}}
    tab = bench.shape_table()
    s1, s2, p1, p2 = bench.pairs(args.pairs, len(tab["type"]), seed=1000)
    model["classes"]["polytope-polytope (bench configs[3])"] = fit(c_oracle.op_counts(tab, s1, s2, p1, p2))
    mt = bench.mixed_table()
    ms1, ms2, mp1, mp2 = bench.mixed_pairs(mt, 40 * args.pairs, seed=0)
    k1, k2 = mt["type"][ms1], mt["type"][ms2]
    for a in range(6):
        for b in range(6):
            if a > 2 and b > 2:
                continue
            sel = np.flatnonzero((k1 == a) & (k2 == b))[:args.pairs]
            oc = c_oracle.op_counts(mt, ms1[sel], ms2[sel], mp1[sel], mp2[sel])
            model["classes"][f"{NAMES[a]}-{NAMES[b]}"] = fit(oc)
    out = os.path.join(REPO, "profiles", "flop_model.json")
    with open(out, "w") as f:
        json.dump(model, f, indent=1)
    print(json.dumps(model["classes"]["polytope-polytope (bench configs[3])"]))
    print("->", out)


if __name__ == "__main__":
    main()
