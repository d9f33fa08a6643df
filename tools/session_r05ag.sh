#!/bin/bash
# Round-5 session AG: polygon x polytope unit (p61) under max-ilp in the product -- GPU suite
# (oracle parity on every pair of the 1M mixed set, codegen twin), the two classes, the 1M mixed step
O=gpurun_out/r05_ag
mkdir -p $O
CB="python3 tools/class_bench.py --small 0 --classes polygon-polytope,polytope-polygon,capsule-polytope"
OUT=$O tools/gpu_session.sh \
  "tests|900|python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread" \
  "cls_a|300|$CB" "mixed_a|200|python3 tools/mixed_buckets.py --steps 60" \
  "cls_b|300|$CB" "mixed_b|200|python3 tools/mixed_buckets.py --steps 60"
