#!/usr/bin/env python3
"""GPU vs C-oracle agreement on random shape tables (tests/stress_shapes.py): per pair
class and row bucket, status / iteration-count agreement and worst alpha / gradient error.
Usage: python3 tools/stress_probe.py [--pairs 200000] [--seed 0]"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [REPO, os.path.join(REPO, "dcol-trajectory-optimization_amd"), os.path.join(REPO, "tests")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=200_000)
    ap.add_argument("--seed", type=int, default=0)
    args = ap.parse_args()
    from dcol_amd import Engine, spec_from_arrays
    from oracle import c_oracle
    from stress_shapes import random_pairs, random_table
    rng = np.random.default_rng(args.seed)
    tab = random_table(rng)
    s1, s2, p1, p2 = random_pairs(rng, tab, args.pairs)
    eng = Engine(device=0)
    ids = np.array([eng.register(spec_from_arrays(tab, k)) for k in range(len(tab["type"]))], np.int32)
    res = eng.solve_host(ids[s1], ids[s2], p1, p2, grad="fd")
    ref = c_oracle.run_batch(tab, s1, s2, p1, p2, want_grad=True, threads=16)
    st_eq = res.status == ref["status"]
    ok = (ref["status"] == 0) & st_eq
    it_eq = res.iters[ok] == ref["iters"][ok]
    ea = np.abs(res.alpha[ok] - ref["alpha"][ok]) / np.maximum(np.abs(ref["alpha"][ok]), 1e-12)
    eg = np.abs(res.grad[ok] - ref["grad"][ok]).max(1) / np.maximum(np.abs(ref["grad"][ok]).max(1), 1.0)
    rows = tab["nh"][s1] + tab["nh"][s2]
    out = {"pairs": args.pairs, "status_equal": float(st_eq.mean()), "status_mismatch": int((~st_eq).sum()),
           "statuses": {int(k): int(v) for k, v in zip(*np.unique(ref["status"], return_counts=True))},
           "iters_equal": float(it_eq.mean()), "alpha_rel_max": float(ea.max()), "grad_max": float(eg.max()),
           "alpha_rel_p999": float(np.quantile(ea, 0.999)), "grad_p999": float(np.quantile(eg, 0.999)),
           "rows_max": int(rows.max())}
    if (~st_eq).any():
        i = np.flatnonzero(~st_eq)[:10]
        out["mismatch_examples"] = [(int(tab["type"][s1[j]]), int(tab["type"][s2[j]]), int(rows[j]),
                                     int(res.status[j]), int(ref["status"][j])) for j in i]
    if not it_eq.all():
        j = np.flatnonzero(ok)[np.flatnonzero(~it_eq)[:10]]
        out["iter_mismatch_examples"] = [(int(tab["type"][s1[k]]), int(tab["type"][s2[k]]), int(rows[k]),
                                          int(res.iters[k]), int(ref["iters"][k])) for k in j]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
