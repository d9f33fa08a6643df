"""Round-3 drift experiment: compare tools/drift_run.py outputs with the
C oracle (this repo's oracle/, test infrastructure) on the two classes that run the (6,1,12)
LPP-2 ball kernel -- polygon-first x polytope (class 40) and polytope-first x polygon (5) --
and with each other bitwise.
Usage: python3 tools/drift_compare.py label=run.npz [label=run.npz ...]"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "dcol-trajectory-optimization_amd")]
import bench  # noqa: E402
from oracle import c_oracle  # noqa: E402

runs = [(a.split("=", 1)[0], np.load(a.split("=", 1)[1])) for a in sys.argv[1:]]
tab = bench.mixed_table()
s1, s2, p1, p2 = bench.mixed_pairs(tab, 1_000_000, seed=0)
idx = runs[0][1]["idx"]
ref = c_oracle.run_batch(tab, s1[idx], s2[idx], p1[idx], p2[idx], want_grad=True, threads=16)
for name, R in runs:
    for c in (40, 5):
        m = (R["cls"] == c) & (ref["status"] == 0)
        rel = np.abs(R["alpha"][m] - ref["alpha"][m]) / np.abs(ref["alpha"][m])
        g = np.abs(R["grad"][m] - ref["grad"][m]).max(1) / np.maximum(np.abs(ref["grad"][m]).max(1), 1)
        print(f"{name:40s} class {c:2d} n {m.sum():6d} alpha rel max {rel.max():.3e} n(>1e-10) {(rel > 1e-10).sum():4d} "
              f"grad max {g.max():.3e} iters equal {bool(np.array_equal(R['iters'][m], ref['iters'][m]))}")
for i in range(len(runs)):
    for j in range(i + 1, len(runs)):
        for c in (40, 5):
            m = runs[i][1]["cls"] == c
            eq = np.mean(runs[i][1]["alpha"][m] == runs[j][1]["alpha"][m])
            print(f"{runs[i][0]} vs {runs[j][0]}: alpha bitwise-equal fraction, class {c}: {eq:.6f}")
