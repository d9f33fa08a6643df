#!/bin/bash
# Round-5 session V: GPU tests on the size-dependent fan-out build, then the driver's command
# (large plans over 2 side streams, small plans over 3) against DCOL_SIDE_STREAMS_LARGE=3.
O=gpurun_out/r05_v
mkdir -p $O
B="python3 bench.py --steps 20 --warmup 5"
OUT=$O tools/gpu_session.sh \
  "tests|600|python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread" \
  "new_a|300|$B" "old_a|300|DCOL_SIDE_STREAMS_LARGE=3 $B" \
  "new_b|300|$B" "old_b|300|DCOL_SIDE_STREAMS_LARGE=3 $B"
