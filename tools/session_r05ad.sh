#!/bin/bash
# Round-5 session AD: EXPERIMENT lane rule -- the one-wave-per-SIMD buckets on one lane
O=gpurun_out/r05_ad
mkdir -p $O
M="python3 tools/mixed_buckets.py --steps 60"
OUT=$O tools/gpu_session.sh "a0|200|$M" "a1|200|DCOL_FANOUT_ASSIGN=1 $M" "b0|200|$M" "b1|200|DCOL_FANOUT_ASSIGN=1 $M" \
  "c1_3|200|DCOL_FANOUT_ASSIGN=1 DCOL_SIDE_STREAMS_LARGE=3 $M" "c0_3|200|DCOL_SIDE_STREAMS_LARGE=3 $M"
