#!/bin/bash
# Round-5 session Y: capsule / cylinder x polytope at two lanes per pair and two waves per SIMD
# (lib_ab: PART (5, 1) buckets (8, 2) / (10, 2) with an LPP-2 WPS-2 copy) against the
# one-lane one-wave product choice and the LPP-2 one-wave copy; class bench, 200k pairs.
O=gpurun_out/r05_y
mkdir -p $O
L=dcol-trajectory-optimization_amd
A="DCOL_LIB=$L/lib_ab/libdcol.so"
C="capsule-polytope,polytope-capsule,cylinder-polytope,polytope-cylinder"
CB="python3 tools/class_bench.py --small 0 --classes $C"
OUT=$O tools/gpu_session.sh \
  "l1_a|300|$A $CB" "l2w2_a|300|$A DCOL_LPP=2 DCOL_WPS=2 $CB" "l2w1_a|300|$A DCOL_LPP=2 DCOL_WPS=1 $CB" \
  "l1_b|300|$A $CB" "l2w2_b|300|$A DCOL_LPP=2 DCOL_WPS=2 $CB" "l2w1_b|300|$A DCOL_LPP=2 DCOL_WPS=1 $CB"
