#!/usr/bin/env python3
"""Cost of a resident one-pair server to a batch plan on the same GPU: the 100k poly x poly
plan (bench configs[3]) timed with HIP events (median of 40 launches) with the table's
server stopped and resident, alternately, three rounds; the drop-in's launch path (a call
with other flags) with the server resident and without it.  The library's A/B knobs act
through the environment (DCOL_PAIR_SERVER_STREAM=normal / high, DCOL_PAIR_SERVER_POLL_SLEEP=<n>,
DCOL_PAIR_SERVER_YIELD=0: the server does not leave when a batch plan launches).
Usage: python3 tools/server_tax.py [--label x]"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(REPO, "dcol-trajectory-optimization_amd"), REPO]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--label", default="")
    a = ap.parse_args()
    os.environ.setdefault("DCOL_PAIR_SERVER_IDLE_US", "30000000")
    import torch
    from bench import pairs, shape_table
    from dcol_amd import Engine, alloc_outputs, spec_from_arrays
    from primitives.misc_primitive_constructor import SphereMRP, create_rect_prism
    eng = Engine(device=0)
    tab = shape_table()
    ids = np.array([eng.register(spec_from_arrays(tab, k)) for k in range(len(tab["type"]))], np.int32)
    box = create_rect_prism(1.0, 2.0, 0.5)
    ball = SphereMRP(0.4)
    box.r, box.p = np.zeros(3), np.array([0.1, -0.2, 0.3])
    ball.r, ball.p = np.array([2.0, 0.5, -0.3]), np.zeros(3)
    eng.solve_pair(ball, box, grad=None)
    B = 100_000
    s1, s2, p1, p2 = pairs(B, len(tab["type"]), seed=3)
    plan = eng.plan(ids[s1], ids[s2], cache=False)
    dev = torch.device("cuda", 0)
    d1 = torch.from_numpy(np.ascontiguousarray(p1.T)).to(dev)
    d2 = torch.from_numpy(np.ascontiguousarray(p2.T)).to(dev)
    out = alloc_outputs(B, dev, want_grad=True, want_contact=False)
    stream = torch.cuda.current_stream(dev)
    run = plan.bind(d1, d2, out, grad="fd", contact=False, stream=stream)

    def timed(n=40):
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
        for x, y in ev:
            x.record(stream)
            run()
            y.record(stream)
        ev[-1][1].synchronize()
        return float(np.median([x.elapsed_time(y) for x, y in ev]))

    for _ in range(60):
        run()
    stream.synchronize()
    t = {"stopped": [], "resident": []}
    for _ in range(3):
        eng.stop_pair_server()
        t["stopped"].append(timed())
        eng.solve_pair(ball, box, grad=None)
        assert eng.pair_server_running()
        t["resident"].append(timed())
        left = not eng.pair_server_running()
    st = eng.pair_stats()
    res = {"label": a.label, "yield": os.environ.get("DCOL_PAIR_SERVER_YIELD", "1"), "server_left_at_launch": left, "stream": os.environ.get("DCOL_PAIR_SERVER_STREAM", "cumask"),
           "poll_sleep": os.environ.get("DCOL_PAIR_SERVER_POLL_SLEEP", "0"), "batch_ms": t,
           "ratio_min": min(t["resident"]) / min(t["stopped"]),
           "server_clock_ghz": st["server_solve_cycles"] / max(st["server_solve_us"], 1e-9) / 1e3}
    lat = {}
    for state in ("resident", "stopped"):
        if state == "stopped":
            eng.stop_pair_server()
            os.environ["DCOL_PAIR_SERVER"] = "0"
        else:
            eng.solve_pair(ball, box, grad=None)
        ts = []
        for _ in range(50):
            t0 = time.perf_counter()
            eng.solve_pair(ball, box, grad="envelope")
            ts.append(time.perf_counter() - t0)
            if state == "resident":
                eng.solve_pair(ball, box, grad=None)
        lat[state] = 1e6 * float(np.median(ts))
    os.environ["DCOL_PAIR_SERVER"] = "1"
    eng.stop_pair_server()
    res["launch_path_us"] = lat
    # queue sharing: the plan on 8 more streams while a server is resident (idle time 3 s): a
    # stream whose hardware queue the server shares waits for the server to leave (~3 s)
    os.environ["DCOL_PAIR_SERVER_IDLE_US"] = "3000000"
    streams = [torch.cuda.Stream(dev) for _ in range(8)]
    eng.solve_pair(ball, box, grad=None)
    waits = []
    for st in streams:
        go = plan.bind(d1, d2, out, grad="fd", contact=False, stream=st)
        t0 = time.perf_counter()
        go()
        st.synchronize()
        waits.append(1e3 * (time.perf_counter() - t0))
    eng.stop_pair_server()
    res["plan_ms_on_8_streams_server_resident"] = waits
    res["hw_queues"] = os.environ.get("GPU_MAX_HW_QUEUES")
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
