#!/bin/bash
# Round-5 session J: the drop-in's per-request device time by phase (stamps build), three
# processes (the device time differs from process to process: 23.7-30.0 us per call this round)
O=gpurun_out/r05_j
mkdir -p $O
L=dcol-trajectory-optimization_amd/lib_stamps/libdcol.so
OUT=$O tools/gpu_session.sh \
  "stamps_p1|200|DCOL_LIB=$L python3 tools/dropin_stamps.py --label p1" \
  "stamps_p2|200|DCOL_LIB=$L python3 tools/dropin_stamps.py --label p2" \
  "stamps_p3|200|DCOL_LIB=$L python3 tools/dropin_stamps.py --label p3" \
  "dropin_prod|200|python3 tools/dropin_ab.py --rounds 2"
