#!/usr/bin/env python3
"""Is one big launch slower per pair than the same pairs as smaller launches in flight on
several streams?  bench.py's kernel_1m (one 1M-pair launch) measures 2.28e9 pair-solves/s,
its pipelined 100k line 2.72e9.  Here the same 1M pairs (bench.py pairs(), seed 7) run as
  one   : one 1M-pair launch,
  chunks: C launches of 1M / C pairs issued round-robin on S streams (same_slice: the first
          1M / C pairs C times -- a working set that stays cache-resident, like bench.py's
          100k batch repeated step after step),
timed with HIP events around the whole batch (median of `reps`, after warm-ups).
Usage: python3 tools/chunk_probe.py [--reps 10]
"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [REPO, os.path.join(REPO, "dcol-trajectory-optimization_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    os.environ["GPU_MAX_HW_QUEUES"] = "8"   # as bench.py: the streams on their own hardware queues
    import torch

    import bench
    from dcol_amd import Engine, alloc_outputs, spec_from_arrays
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    eng = Engine(device=0)
    tab = bench.shape_table()
    ids = np.array([eng.register(spec_from_arrays(tab, k)) for k in range(len(tab["type"]))], np.int32)
    B = 1_000_000
    s1, s2, p1, p2 = bench.pairs(B, len(tab["type"]), seed=7)
    d1 = torch.from_numpy(np.ascontiguousarray(p1.T)).to(dev)
    d2 = torch.from_numpy(np.ascontiguousarray(p2.T)).to(dev)
    main_stream = torch.cuda.current_stream(dev)

    def runner(C, S, same=False):
        streams = [main_stream] + [torch.cuda.Stream(dev) for _ in range(S - 1)]
        n = B // C
        fns = []
        for c in range(C):
            sl = slice(0, n) if same else slice(c * n, (c + 1) * n)   # same: one slice C times (cache-warm)
            plan = eng.plan(ids[s1[sl]], ids[s2[sl]], cache=False)
            a1 = d1[:, sl].contiguous()
            a2 = d2[:, sl].contiguous()
            out = alloc_outputs(n, dev, want_grad=True, want_contact=False)
            fns.append((plan, plan.bind(a1, a2, out, grad="fd", contact=False, stream=streams[c % S]), a1, a2, out))
        fork = torch.cuda.Event()
        joins = [torch.cuda.Event() for _ in streams]

        def run():
            fork.record(main_stream)
            for s in streams[1:]:
                s.wait_event(fork)
            for f in fns:
                f[1]()
            for s, j in zip(streams[1:], joins[1:]):
                j.record(s)
                main_stream.wait_event(j)
        return run, fns

    rows = []
    for C, S, same in ((1, 1, False), (10, 2, False), (10, 2, True), (10, 1, True), (10, 1, False), (5, 2, False)):
        run, keep = runner(C, S, same)
        for _ in range(3):
            run()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.reps)]
        for e0, e1 in ev:
            e0.record(main_stream)
            run()
            e1.record(main_stream)
        torch.cuda.synchronize(dev)
        ms = float(np.median([a.elapsed_time(b) for a, b in ev]))
        row = {"chunks": C, "streams": S, "same_slice": same, "ms": round(ms, 4), "pair_solves_per_s": round(B / (ms * 1e-3) / 1e9, 4)}
        rows.append(row)
        print(json.dumps(row), flush=True)
        del keep


if __name__ == "__main__":
    main()
