#!/usr/bin/env python3
"""Diagnostic: fused vs per-bucket launches of a golden scene plan, mismatches per pair class.
Usage: python3 tools/fused_diff.py [scene_quad.npz]"""
import os
import sys

import numpy as np

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(REPO, "dcol-trajectory-optimization_amd"), os.path.join(REPO, "tests"), REPO]


def main(name):
    import torch
    from dcol_amd import Engine, spec_from_arrays
    d = dict(np.load(os.path.join(REPO, "tests", "golden", name), allow_pickle=False))
    eng = Engine(device=0)
    ids = np.array([eng.register(spec_from_arrays(d, k)) for k in range(len(d["type"]))], np.int32)
    s1, s2 = ids[d["s1"]], ids[d["s2"]]
    fused = eng.plan(s1, s2, cache=False)
    split = eng.plan(s1, s2, cache=False, fuse=False)
    p1 = torch.from_numpy(np.ascontiguousarray(d["pose1"].T)).cuda()
    p2 = torch.from_numpy(np.ascontiguousarray(d["pose2"].T)).cuda()
    a = fused.run(p1, p2, grad="fd")
    b = split.run(p1, p2, grad="fd")
    torch.cuda.synchronize()
    al, bl = a["alpha"].cpu().numpy(), b["alpha"].cpu().numpy()
    if os.environ.get("DUMP"):
        np.savez(os.environ["DUMP"], fused=al, split=bl)
    t1, t2 = d["type"][d["s1"]], d["type"][d["s2"]]
    bad = al != bl
    for c in sorted(set(zip(t1, t2))):
        m = (t1 == c[0]) & (t2 == c[1])
        print("class", c, "pairs", int(m.sum()), "alpha mismatches", int((bad & m).sum()),
              "iters equal", bool(np.all(a["iters"].cpu().numpy()[m] == b["iters"].cpu().numpy()[m])))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "scene_quad.npz")
