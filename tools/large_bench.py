#!/usr/bin/env python3
"""Throughput of the many-faced row buckets (48 / 64 / 128 orthant rows, 8-16 lanes per
pair): random k-face polytopes (6 box normals + k - 6 random ones, as
tests/golden/gen_golden.py: rand_polytope) against a box and against each other, B pairs
per class, poses as bench.py configs[3], FD gradients, one launch at a time (HIP events).
Each class is also checked against the C oracle on its first 512 pairs (status and
iteration counts equal, alpha within 1e-6 rel).
Usage: python3 tools/large_bench.py [--pairs 100000] [--reps 10]
"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "dcol-trajectory-optimization_amd"))


def polytope_table(faces, seed=5):
    rng = np.random.default_rng(seed)
    A_rows, b_rows, nh, off = [], [], [], []
    for k in faces:
        A = np.vstack([np.eye(3), -np.eye(3), rng.normal(size=(k - 6, 3))])
        A /= np.linalg.norm(A, axis=1, keepdims=True)
        off.append(len(b_rows))
        A_rows += list(A)
        b_rows += list(rng.uniform(0.4, 1.3, k))
        nh.append(k)
    S = len(faces)
    return {"type": np.zeros(S, np.int32), "nh": np.array(nh, np.int32), "A_off": np.array(off, np.int32),
            "A_pool": np.array(A_rows), "b_pool": np.array(b_rows), "params": np.zeros((S, 4)),
            "r_offset": np.zeros((S, 3)), "Q_offset": np.tile(np.eye(3), (S, 1, 1))}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=100_000)
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    import torch
    from dcol_amd import Engine, alloc_outputs, spec_from_arrays
    from oracle import c_oracle
    faces = [6, 20, 30, 40, 58]
    tab = polytope_table(faces)
    eng = Engine(device=0)
    ids = np.array([eng.register(spec_from_arrays(tab, k)) for k in range(len(faces))], np.int32)
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(0)
    B = args.pairs
    for a, b in ((1, 0), (2, 0), (3, 0), (4, 0), (2, 1), (3, 2), (4, 3), (4, 4)):
        s1 = np.full(B, a, np.int32)
        s2 = np.full(B, b, np.int32)
        p1 = np.hstack([rng.uniform(-3, 3, (B, 3)), rng.uniform(-1, 1, (B, 3))])
        p2 = np.hstack([rng.uniform(-3, 3, (B, 3)), rng.uniform(-1, 1, (B, 3))])
        plan = eng.plan(ids[s1], ids[s2])
        d1 = torch.from_numpy(np.ascontiguousarray(p1.T)).to(dev)
        d2 = torch.from_numpy(np.ascontiguousarray(p2.T)).to(dev)
        out = alloc_outputs(B, dev, want_grad=True, want_contact=False)
        stream = torch.cuda.current_stream(dev)
        step = plan.bind(d1, d2, out, grad="fd", contact=False, stream=stream)
        for _ in range(3):
            step()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.reps)]
        for e0, e1 in ev:
            e0.record(stream)
            step()
            e1.record(stream)
        torch.cuda.synchronize(dev)
        ms = float(np.mean([e0.elapsed_time(e1) for e0, e1 in ev]))
        st = out["status"].cpu().numpy()
        it = out["iters"].cpu().numpy()
        al = out["alpha"].cpu().numpy()
        n = 512
        ref = c_oracle.run_batch(tab, s1[:n], s2[:n], p1[:n], p2[:n], want_grad=True, threads=16)
        ok = ref["status"] == 0
        print(json.dumps({
            "class": f"poly{faces[a]}-poly{faces[b]}", "orthant_rows": faces[a] + faces[b], "pairs": B,
            "kernel_ms": ms, "pair_solves_per_s": B / (ms * 1e-3), "ok_frac": float(np.mean(st == 0)),
            "iters_mean": float(it[st == 0].mean()), "iters_max": int(it.max()),
            "oracle_status_equal": bool(np.array_equal(st[:n], ref["status"])),
            "oracle_iters_equal": float(np.mean(it[:n][ok] == ref["iters"][ok])),
            "oracle_alpha_ok": bool(np.all(np.abs(al[:n][ok] - ref["alpha"][ok]) <= 1e-6 * np.abs(ref["alpha"][ok]) + 1e-12)),
        }), flush=True)


if __name__ == "__main__":
    main()
