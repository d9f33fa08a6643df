#!/usr/bin/env python3
"""A/B of two builds of the library on the same workloads (run once per build, DCOL_LIB
selecting the build): the 1M mixed plan (bench.py --workload mixed1m pairs) and the 100k
poly x poly plan, outputs saved for a bitwise comparison.
Usage: DCOL_LIB=<lib> python3 tools/lib_ab.py --save out.npz
       python3 tools/lib_ab.py --compare a.npz b.npz"""
import argparse
import os
import sys

import numpy as np

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(REPO, "dcol-trajectory-optimization_amd"), REPO]


def run(path):
    import bench
    from dcol_amd import Engine, spec_from_arrays
    out = {}
    for name, tab, gen in (("mixed", bench.mixed_table(), lambda t: bench.mixed_pairs(t, 1_000_000, seed=0)),
                           ("poly", bench.shape_table(), lambda t: bench.pairs(100_000, len(t["type"]), seed=1000))):
        s1, s2, p1, p2 = gen(tab)
        eng = Engine(device=0)
        ids = np.array([eng.register(spec_from_arrays(tab, j)) for j in range(len(tab["type"]))], np.int32)
        r = eng.solve_host(ids[s1], ids[s2], p1, p2, grad="fd", contact=True)
        for k in ("alpha", "contact", "grad", "iters", "status"):
            out[f"{name}_{k}"] = getattr(r, k)
    np.savez(path, lib=os.environ.get("DCOL_LIB", "default"), **out)
    print("saved", path, {k: v.shape for k, v in out.items() if k.endswith("alpha")})


def compare(a, b):
    A, B = np.load(a), np.load(b)
    bad = 0
    for k in A.files:
        if k == "lib":
            continue
        x, y = A[k], B[k]
        same = x.view(np.uint8).tobytes() == y.view(np.uint8).tobytes()
        if not same:
            bad += 1
            d = np.flatnonzero((x != y) & ~(np.isnan(x) & np.isnan(y))) if x.dtype.kind == "f" else np.flatnonzero(x != y)
            print(f"{k}: {d.size} differing entries (first {d[:5].tolist()})")
    print(f"compare {A['lib']} vs {B['lib']}: {'BITWISE EQUAL' if not bad else f'{bad} arrays differ'}")
    return bad


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--save")
    ap.add_argument("--compare", nargs=2)
    a = ap.parse_args()
    if a.save:
        run(a.save)
    if a.compare:
        sys.exit(1 if compare(*a.compare) else 0)
