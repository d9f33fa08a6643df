#!/bin/bash
# Round-5 session AA: lane assignment of the 1M mixed plan's buckets (EXPERIMENT knob
# DCOL_FANOUT_ASSIGN: 0 longest-processing-time greedy (default), 1 round robin, 2 snake)
O=gpurun_out/r05_aa
mkdir -p $O
M="python3 tools/mixed_buckets.py --steps 60"
OUT=$O tools/gpu_session.sh "a0|200|$M" "a1|200|DCOL_FANOUT_ASSIGN=1 $M" "a2|200|DCOL_FANOUT_ASSIGN=2 $M" \
  "b0|200|$M" "b1|200|DCOL_FANOUT_ASSIGN=1 $M" "b2|200|DCOL_FANOUT_ASSIGN=2 $M"
