#!/bin/bash
# Round-5 session AH: the N = 6, NSOC = 2 PART unit split by SOC flavour (dense copies under
# max-ilp) -- GPU suite, the four classes of the unit, the 1M mixed step
O=gpurun_out/r05_ah
mkdir -p $O
CB="python3 tools/class_bench.py --small 0 --classes cone-polygon,polygon-cone,polygon-sphere,sphere-polygon"
OUT=$O tools/gpu_session.sh \
  "tests|900|python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread" \
  "cls_a|300|$CB" "mixed_a|200|python3 tools/mixed_buckets.py --steps 60" \
  "cls_b|300|$CB" "mixed_b|200|python3 tools/mixed_buckets.py --steps 60"
