#!/bin/bash
# Round-5 session S: the 1M mixed plan's step time (synchronised steps, HIP events) against
# the number of fan-out streams and hardware queues.
O=gpurun_out/r05_s
mkdir -p $O
M="python3 tools/mixed_buckets.py --steps 60"
OUT=$O tools/gpu_session.sh \
  "q4s3_a|200|$M" \
  "q8s3_a|200|GPU_MAX_HW_QUEUES=8 $M" \
  "q8s5_a|200|GPU_MAX_HW_QUEUES=8 DCOL_SIDE_STREAMS=5 $M" \
  "q8s7_a|200|GPU_MAX_HW_QUEUES=8 DCOL_SIDE_STREAMS=7 $M" \
  "q4s2_a|200|DCOL_SIDE_STREAMS=2 $M" \
  "q4s3_b|200|$M" \
  "q8s3_b|200|GPU_MAX_HW_QUEUES=8 $M" \
  "q8s5_b|200|GPU_MAX_HW_QUEUES=8 DCOL_SIDE_STREAMS=5 $M" \
  "q8s7_b|200|GPU_MAX_HW_QUEUES=8 DCOL_SIDE_STREAMS=7 $M" \
  "q4s2_b|200|DCOL_SIDE_STREAMS=2 $M"
