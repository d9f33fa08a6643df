#!/usr/bin/env python3
"""A/B timing of dcol_altro_backward (the Riccati sweep) between builds of libdcol_altro.so
on one captured quadrotor input (tools/bw_in.npz).  Usage: riccati_ab.py lib1.so lib2.so ..."""
import os
import sys
import time

import numpy as np

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dcol-trajectory-optimization_amd")]
from altro import _native  # noqa: E402

d = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "bw_in.npz"))
st = [d[f"s{i}"] for i in range(6)]
res = {}
for rnd in range(3):
    for path in sys.argv[1:]:
        _native._lib = None
        _native.load(path)
        _native.backward(d["A"], d["B"], *st, 1e-6)
        t0 = time.perf_counter()
        for _ in range(500):
            _native.backward(d["A"], d["B"], *st, 1e-6)
        res.setdefault(path, []).append(1e3 * (time.perf_counter() - t0) / 500)
for p, v in res.items():
    print(os.path.basename(p), "backward ms (min of 3):", round(min(v), 4), [round(x, 4) for x in v])
