#!/bin/bash
# Round-5 session AB: one-pair latency of the quadrotor pairs per lanes-per-pair choice
# (tools/dropin_latency.py plan_run / c_call paths; DCOL_LPP forces the bucket's LPP)
O=gpurun_out/r05_ab
mkdir -p $O
D="python3 tools/dropin_latency.py --calls 300"
OUT=$O tools/gpu_session.sh "def|200|$D" "l1|200|DCOL_LPP=1 $D" "l2|200|DCOL_LPP=2 $D" "l4|200|DCOL_LPP=4 $D" "l8|200|DCOL_LPP=8 $D" "def2|200|$D"
