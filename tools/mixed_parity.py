#!/usr/bin/env python3
"""Diagnostic: GPU engine vs the C restatement (oracle/, test infrastructure) on the first K
pairs of the mixed 1M workload (bench.py --workload mixed1m); prints the worst alpha /
gradient deviations with their pair class and Newton iteration counts.
Usage: python3 tools/mixed_parity.py [K]"""
import os
import sys

import numpy as np

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(REPO, "dcol-trajectory-optimization_amd"), REPO]

import bench  # noqa: E402


def main(k):
    from dcol_amd import Engine, spec_from_arrays
    from oracle import c_oracle
    tab = bench.mixed_table()
    s1, s2, p1, p2 = bench.mixed_pairs(tab, 1_000_000, seed=0)
    eng = Engine(device=0)
    ids = np.array([eng.register(spec_from_arrays(tab, j)) for j in range(len(tab["type"]))], np.int32)
    full = eng.solve_host(ids[s1], ids[s2], p1, p2, grad="fd")   # the whole 1M plan (throughput variants)
    s1, s2, p1, p2 = s1[:k], s2[:k], p1[:k], p2[:k]
    res = type(full)(*(None if a is None else a[:k] for a in (full.alpha, full.contact, full.grad, full.iters, full.status)))
    ref = c_oracle.run_batch(tab, s1, s2, p1, p2, want_grad=True, threads=16)
    ok = (ref["status"] == 0) & (res.status == 0)
    print("status equal", bool(np.array_equal(res.status, ref["status"])),
          "iters equal frac", float(np.mean(res.iters[ok] == ref["iters"][ok])))
    ea = np.abs(res.alpha - ref["alpha"]) / np.abs(ref["alpha"])
    eg = np.abs(res.grad - ref["grad"]).max(1) / np.maximum(np.abs(ref["grad"]).max(1), 1)
    for name, e in (("alpha", ea), ("grad", eg)):
        e = np.where(ok, e, 0)
        for i in np.argsort(-e)[:5]:
            print(name, "pair", int(i), "class", int(tab["type"][s1[i]]), int(tab["type"][s2[i]]), "rel err %.3e" % e[i],
                  "iters", int(res.iters[i]), int(ref["iters"][i]), "alpha %.6g" % ref["alpha"][i])


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 16384)
