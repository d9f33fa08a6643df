#!/usr/bin/env python3
"""Where the drop-in's per-call latency goes (bench.py `dropin`): one quadrotor pair kind at
a time, timed on the host clock over many calls --
  python   : proximity_mrp / proximity_gradient (the drop-in, Python + C + GPU)
  device   : of those, the one-pair server's request-to-answer time on the device
  batch_host: the same pair through solve_objects -> dcol_prox_batch_host (round 2's path)
  c_call   : dcol_prox_pair through ctypes with pre-built arguments (C + GPU)
  plan_run : the same one-pair plan on device-resident poses, launch + hipStreamSynchronize
             through torch (no mapped memory, no staging)
  launch   : an empty torch kernel + synchronize (the launch / completion floor)
Usage: python3 tools/dropin_latency.py [--calls 2000]
"""
import argparse
import ctypes
import os
import sys
import time

import numpy as np

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [REPO, os.path.join(REPO, "dcol-trajectory-optimization_amd")]


def best_us(fn, calls):
    fn()
    t = []
    for _ in range(5):
        t0 = time.perf_counter()
        for _ in range(calls):
            fn()
        t.append((time.perf_counter() - t0) / calls * 1e6)
    return min(t)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=2000)
    args = ap.parse_args()
    import torch
    from altro import systems
    from dcol_amd import _lib
    from dcol_amd.engine import default_engine
    from proximity.proximity import proximity_mrp
    from proximity.proximity_gradient import proximity_gradient
    params, X, U = systems.initialize("quadrotor")
    vic, obs = params["P_vic"], params["P_obs"]
    x = np.asarray(params["Xref"], dtype=np.float64).reshape(-1, int(params["nx"]))[50]
    vic.r, vic.p = np.array(x[0:3]), np.array(x[6:9])
    eng = default_engine()
    lib = _lib.load()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    z = torch.zeros(1, device=dev)
    floor = best_us(lambda: (z.add_(1), torch.cuda.synchronize()), args.calls)
    print({"launch_floor_us": round(floor, 2)}, flush=True)
    for o in obs:
        kind = type(o).__name__
        row = {"obstacle": kind}
        s0 = eng.pair_stats()
        row["python_mrp_us"] = best_us(lambda: proximity_mrp(vic, o), args.calls)
        s1 = eng.pair_stats()
        row["python_grad_us"] = best_us(lambda: proximity_gradient(vic, o), args.calls)
        s2 = eng.pair_stats()
        for key, a, b in (("device_mrp_us", s0, s1), ("device_grad_us", s1, s2)):
            n = b["served"] - a["served"]   # one-pair server: request-to-answer time on the device
            if n > 0:
                row[key] = (b["server_solve_us"] - a["server_solve_us"]) / n
        # round 2's per-call path: a transient plan + pageable staging (dcol_prox_batch_host)
        row["batch_host_grad_us"] = best_us(lambda: eng.solve_objects([vic], [o], grad="fd", contact=False), args.calls)
        s1, s2 = eng.register_object(vic), eng.register_object(o)
        pose = np.concatenate([vic.r, vic.p, o.r, o.p]).astype(np.float64)
        out = np.empty(16)
        ints = np.empty(2, np.int32)
        P = lambda a, off=0: ctypes.c_void_p(a.ctypes.data + off)  # noqa: E731
        cargs = (eng.table.handle, s1, s2, P(pose), P(pose, 48), 1e-6, 50, _lib.GRAD_FD, P(out), None, P(out, 8),
                 P(ints), P(ints, 4))
        row["c_call_grad_us"] = best_us(lambda: lib.dcol_prox_pair(*cargs), args.calls)
        plan = eng.plan(np.array([s1]), np.array([s2]), cache=False)
        p1 = torch.from_numpy(pose[:6].reshape(6, 1).copy()).to(dev)
        p2 = torch.from_numpy(pose[6:].reshape(6, 1).copy()).to(dev)
        from dcol_amd import alloc_outputs
        o_ = alloc_outputs(1, dev, True, False)
        run = plan.bind(p1, p2, o_, grad="fd", stream=torch.cuda.current_stream(dev))
        row["plan_run_grad_us"] = best_us(lambda: (run(), torch.cuda.synchronize()), args.calls)
        print({k: (round(v, 2) if isinstance(v, float) else v) for k, v in row.items()}, flush=True)


if __name__ == "__main__":
    main()
