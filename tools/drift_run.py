"""Round-3 drift experiment: commit 326f844 rebuilt with the (6,1,12)
LPP-2 ball kernel as polygon x box's throughput variant -- (a) as it was, (b) with the DPP
reads bound_ctrl-ed (no undefined source register) -- solving the 1M mixed workload.
Usage: python3 tools/drift_run.py <which> <out.npz>  (drift326/<which>: a copy of that build of
the package and its library, git-ignored; a = as it was, b = bound_ctrl DPP, c = a with
-amdgpu-waitcnt-forcezero)"""
import os
import sys

import numpy as np

HERE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "drift326")
which, out = sys.argv[1], sys.argv[2]
sys.path[:0] = [os.path.join(HERE, which, "dcol-trajectory-optimization_amd"), os.path.join(HERE, which)]
import bench  # noqa: E402
from dcol_amd import Engine, spec_from_arrays  # noqa: E402

tab = bench.mixed_table()
s1, s2, p1, p2 = bench.mixed_pairs(tab, 1_000_000, seed=0)
eng = Engine(device=0)
ids = np.array([eng.register(spec_from_arrays(tab, k)) for k in range(len(tab["type"]))], np.int32)
r = eng.solve_host(ids[s1], ids[s2], p1, p2, grad="fd")
cls = tab["type"][s1] * 8 + tab["type"][s2]
m = (cls == 40) | (cls == 5)
np.savez(out, idx=np.flatnonzero(m), cls=cls[m], alpha=r.alpha[m], grad=r.grad[m], iters=r.iters[m], status=r.status[m])
print(which, "solved", int(m.sum()), "class-40/5 pairs")
