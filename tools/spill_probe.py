#!/usr/bin/env python3
"""Diagnostic for the (N=6, NSOC=1, OMAX=12) ball kernel at LPP 2 (polygon x box): solve a
polygon x box batch large enough for the throughput variant with the library named by
DCOL_LIB (default: the in-tree one) and save the outputs, so that runs with different
libraries / DCOL_LPP / DCOL_NO_BALL can be compared with each other and with the C oracle
on the host (tools/spill_probe.py compare ...).

  gpu:     DCOL_LIB=probe/lib/libdcol.so python3 tools/spill_probe.py run <tag> [B]
  host:    python3 tools/spill_probe.py compare <tag> [<tag> ...]
"""
import os
import sys

import numpy as np

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(REPO, "dcol-trajectory-optimization_amd"), REPO]
OUT = os.path.join(REPO, "gpurun_out")

import bench  # noqa: E402


def batch(B, seed=5):
    tab = bench.mixed_table()
    rng = np.random.default_rng(seed)
    poly = np.flatnonzero(tab["type"] == 5)
    box = np.flatnonzero(tab["type"] == 0)
    first_poly = rng.random(B) < 0.5
    a = rng.choice(poly, B)
    b = rng.choice(box, B)
    s1 = np.where(first_poly, a, b).astype(np.int32)
    s2 = np.where(first_poly, b, a).astype(np.int32)
    pose1 = np.hstack([rng.uniform(-3, 3, (B, 3)), rng.uniform(-1, 1, (B, 3))])
    pose2 = np.hstack([rng.uniform(-3, 3, (B, 3)), rng.uniform(-1, 1, (B, 3))])
    return tab, s1, s2, pose1, pose2


def run(tag, B):
    from dcol_amd import Engine, spec_from_arrays
    tab, s1, s2, p1, p2 = batch(B)
    eng = Engine(device=0)
    ids = np.array([eng.register(spec_from_arrays(tab, k)) for k in range(len(tab["type"]))], np.int32)
    plan = eng.plan(ids[s1], ids[s2])
    res = eng.solve_host(ids[s1], ids[s2], p1, p2, grad="fd")
    os.makedirs(OUT, exist_ok=True)
    np.savez_compressed(os.path.join(OUT, f"probe_{tag}.npz"), alpha=res.alpha, grad=res.grad, iters=res.iters,
             status=res.status, launches=plan.num_launches)
    print(tag, "B", B, "launches", plan.num_launches, "status counts", np.unique(res.status, return_counts=True))


def compare(tags):
    from oracle import c_oracle
    rs = {t: dict(np.load(os.path.join(OUT, f"probe_{t}.npz"))) for t in tags}
    B = len(rs[tags[0]]["alpha"])
    tab, s1, s2, p1, p2 = batch(B)
    ref = c_oracle.run_batch(tab, s1, s2, p1, p2, want_grad=True, threads=8)
    ok = ref["status"] == 0
    for t, r in rs.items():
        e_a = np.where(ok, np.abs(r["alpha"] - ref["alpha"]) / np.abs(ref["alpha"]), 0)
        e_g = np.where(ok, np.abs(r["grad"] - ref["grad"]).max(1) / np.maximum(np.abs(ref["grad"]).max(1), 1), 0)
        print(f"{t}: status equal {np.array_equal(r['status'], ref['status'])}, iters equal "
              f"{np.mean(r['iters'][ok] == ref['iters'][ok]):.6f}, alpha rel max {e_a.max():.3e} "
              f"(> 1e-9: {int((e_a > 1e-9).sum())}), grad max {e_g.max():.3e} (> 1e-6: {int((e_g > 1e-6).sum())})")
        for i in np.argsort(-e_a)[:3]:
            print(f"   pair {i}: alpha err {e_a[i]:.3e} grad err {e_g[i]:.3e} iters {r['iters'][i]} "
                  f"ref {ref['iters'][i]} alpha {ref['alpha'][i]:.6g} s1 type {tab['type'][s1[i]]}")
    for i, t in enumerate(tags):
        for u in tags[i + 1:]:
            a, b = rs[t], rs[u]
            same = (a["alpha"] == b["alpha"]) | (np.isnan(a["alpha"]) & np.isnan(b["alpha"]))
            print(f"{t} vs {u}: alpha bitwise equal on {same.mean():.6f}")


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 100_000)
    else:
        compare(sys.argv[2:])
