#!/bin/bash
# Round-5 session U: two side streams (the new default) against three, the driver's command
# (the default line: 100k section, mixed1m section, ALTRO, drop-in), interleaved.
O=gpurun_out/r05_u
mkdir -p $O
B="python3 bench.py --steps 20 --warmup 5"
OUT=$O tools/gpu_session.sh \
  "s2_a|300|$B" "s3_a|300|DCOL_SIDE_STREAMS=3 $B" \
  "s2_b|300|$B" "s3_b|300|DCOL_SIDE_STREAMS=3 $B"
