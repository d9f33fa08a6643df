#!/bin/bash
# Round-5 session Z: the 1M mixed step with the capsule / cylinder x polytope buckets at two
# lanes per pair and two waves per SIMD (lib_ab) against the product's one-lane one-wave copies
O=gpurun_out/r05_z
mkdir -p $O
L=dcol-trajectory-optimization_amd
A="DCOL_LIB=$L/lib_ab/libdcol.so"
M="python3 tools/mixed_buckets.py --steps 60"
OUT=$O tools/gpu_session.sh "ab_a|200|$A $M" "base_a|200|$M" "ab_b|200|$A $M" "base_b|200|$M" "ab_c|200|$A $M" "base_c|200|$M"
