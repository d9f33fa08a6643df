#!/usr/bin/env python3
"""configs[4]'s per-rank regime on one GPU: rank 0's class-balanced shard of the 1M mixed
batch at world N (dcol_amd.dist.shard_indices, the shard bench.py's mixed1m gives rank 0),
solved alone, K steps back to back on one stream (HIP events around the region), for
N in --worlds.  Prints one JSON line per shard: ms per step, the ratio (1M ms / N) / shard ms
(1.0 = linear), the plan's launches / streams / buckets.

  python tools/shard_bench.py [--worlds 1,2,4,8] [--steps 40] [--buckets]
  python tools/shard_bench.py --sweep      # the same in one child process per plan-policy
                                           # environment (DCOL_* A/B), sequentially
"""
import argparse
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [ROOT, os.path.join(ROOT, "dcol-trajectory-optimization_amd")]

SWEEP = [   # (name, environment, extra arguments)
    ("default", {}, []),
    ("fanout3", {"DCOL_SIDE_STREAMS_LARGE": "3"}, []),
    ("fanout7", {"DCOL_SIDE_STREAMS": "7", "DCOL_SIDE_STREAMS_LARGE": "7"}, []),
    ("serial", {"DCOL_NO_FANOUT": "1"}, []),
    ("lat_per_launch", {"DCOL_LATENCY_PER_LAUNCH": "1"}, []),
    # plans below 500k lanes (the 125k / 250k shards) as small plans: latency configurations,
    # one fused launch (segments longest first / in key order), or fanned out unfused
    ("small_fused", {"DCOL_SMALL_PLAN_LANES": "500000"}, []),
    ("small_fused_keyorder", {"DCOL_SMALL_PLAN_LANES": "500000", "DCOL_FUSED_ORDER": "0"}, []),
    ("small_nofuse", {"DCOL_SMALL_PLAN_LANES": "500000"}, ["--no-fuse"]),
    # the packed launch (dcol_kernels_packed.hip) by threshold: off, the default (8 x 64 x
    # SIMDs lanes), up to the 500k shard, every plan
    ("pack_off", {"DCOL_PACK_LANES": "0"}, []),
    ("pack_1m", {"DCOL_PACK_LANES": "1000000"}, []),
    ("pack_all", {"DCOL_PACK_LANES": "100000000"}, []),
    ("pack_keyorder", {"DCOL_FUSED_ORDER": "0"}, []),
    ("small_fanout", {"DCOL_SMALL_FANOUT": "1"}, []),
]


def measure(worlds, steps, warmup, show_buckets, hwq, fuse=True):
    import torch

    import bench
    from dcol_amd import Engine, alloc_outputs, spec_from_arrays
    from dcol_amd.dist import shard_indices
    dev = torch.device("cuda", 0)
    torch.zeros(1, device=dev)
    B = 1_000_000
    tab = bench.mixed_table()
    s1, s2, p1, p2 = bench.mixed_pairs(tab, B, seed=0)
    cost = tab["type"][s1] * 8 + tab["type"][s2]
    eng = Engine(device=0)
    ids = np.array([eng.register(spec_from_arrays(tab, k)) for k in range(len(tab["type"]))], np.int32)
    stream = torch.cuda.current_stream(dev)
    res = []
    ref = None
    for w in worlds:
        mine = shard_indices(B, 0, w, cost)
        plan = eng.plan(ids[s1[mine]], ids[s2[mine]], cache=False, fuse=fuse)
        d1 = torch.from_numpy(np.ascontiguousarray(p1[mine].T)).to(dev)
        d2 = torch.from_numpy(np.ascontiguousarray(p2[mine].T)).to(dev)
        out = alloc_outputs(len(mine), dev, want_grad=True, want_contact=False)
        run = plan.bind(d1, d2, out, grad="fd", contact=False, stream=stream)
        bench.clock_settle(run, stream, dev, None, 30.0)
        for _ in range(warmup):
            run()
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(steps):
            run()
        e1.record(stream)
        torch.cuda.synchronize(dev)
        ms = e0.elapsed_time(e1) / steps
        # one step at a time (synchronised): the latency a serial step of bench.py sees
        one = []
        for _ in range(10):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            run()
            b.record(stream)
            torch.cuda.synchronize(dev)
            one.append(a.elapsed_time(b))
        st = out["status"].cpu().numpy()
        it = out["iters"].cpu().numpy()
        r = {"world": w, "pairs": int(len(mine)), "ms_per_step": ms, "ms_one_step": float(np.median(one)),
             "pair_solves_per_s": len(mine) / (ms * 1e-3), "launches": plan.num_launches,
             "streams": plan.num_streams, "buckets": plan.num_buckets, "form": plan.launch_form, "iters_mean": float(it[st == 0].mean()),
             "hw_queues": hwq}
        if show_buckets:
            r["bucket_list"] = [(b["N"], b["nsoc"], b["omax"], b["lpp"], b["oe"], b["flags"], b["pairs"])
                                for b in plan.buckets() if b["kind"] == "solve"]
        # parity: the shard's results against the 1M plan's (no cross-pair arithmetic: bitwise)
        if ref is None:
            ref = {"mine": mine, "alpha": out["alpha"].cpu().numpy(), "iters": it}
        else:
            pos = np.searchsorted(ref["mine"], mine)
            r["bitwise_vs_first"] = bool(np.array_equal(out["alpha"].cpu().numpy(), ref["alpha"][pos]) and
                                         np.array_equal(it, ref["iters"][pos]))
        res.append(r)
        del plan, d1, d2, out, run
    base = next((r for r in res if r["world"] == 1), None)
    for r in res:
        if base is not None:
            r["linear_frac"] = base["ms_per_step"] / r["world"] / r["ms_per_step"]
        print(json.dumps(r), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--buckets", action="store_true")
    ap.add_argument("--sweep", action="store_true")
    ap.add_argument("--no-fuse", action="store_true", help="plans with DCOL_PLAN_NO_FUSE")
    ap.add_argument("--only", default="", help="--sweep: comma-separated names of SWEEP entries")
    ap.add_argument("--hw-queues", type=int, default=8, help="GPU_MAX_HW_QUEUES (bench.py's default)")
    a = ap.parse_args()
    if a.sweep:
        names = set(a.only.split(",")) if a.only else None
        for name, env, extra in SWEEP:
            if names and name not in names:
                continue
            e = dict(os.environ, GPU_MAX_HW_QUEUES=str(a.hw_queues), **env)
            print(json.dumps({"config": name, "env": env}), flush=True)
            cmd = [sys.executable, os.path.abspath(__file__), "--worlds", a.worlds, "--steps", str(a.steps),
                   "--warmup", str(a.warmup), "--hw-queues", str(a.hw_queues)] + (["--buckets"] if a.buckets else []) + extra
            rc = subprocess.call(cmd, env=e)
            if rc != 0:
                sys.exit(rc)
        return
    os.environ.setdefault("GPU_MAX_HW_QUEUES", str(a.hw_queues))
    measure([int(x) for x in a.worlds.split(",")], a.steps, a.warmup, a.buckets, os.environ["GPU_MAX_HW_QUEUES"],
            fuse=not a.no_fuse)


if __name__ == "__main__":
    main()
