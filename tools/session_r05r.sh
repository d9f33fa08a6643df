#!/bin/bash
# Round-5 session R: the 1M mixed plan's buckets and their kernel times alone (one stream,
# DCOL_NO_FANOUT) against the four-stream fan-out -- rocprofv3 kernel traces of synchronised
# steps (tools/mixed_buckets.py --steps).
O=gpurun_out/r05_r
mkdir -p $O
M="python3 tools/mixed_buckets.py --steps 30"
OUT=$O tools/gpu_session.sh \
  "plain|200|$M" \
  "serial|300|DCOL_NO_FANOUT=1 rocprofv3 --kernel-trace -f csv -d $O/serial -o run -- $M" \
  "fanout|300|rocprofv3 --kernel-trace -f csv -d $O/fanout -o run -- $M"
