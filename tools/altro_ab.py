import json, os, sys
sys.path.insert(0, "."); sys.path.insert(0, "dcol-trajectory-optimization_amd")
import bench
r = bench.altro_section()
print(json.dumps({k: {"ms_per_iter": v["ms_per_iter"], "prox_ms_per_iter": v["prox_ms_per_iter"], "iters": v["iterations"], "conv": v["converged"]} for k, v in r["systems"].items()}))
