#!/bin/bash
# Round-5 session AI: every unit under max-ilp with the product's LDS rows (lib_ab) against
# the product (per-unit schedule) -- the classes of the default-schedule units
O=gpurun_out/r05_ai
mkdir -p $O
L=dcol-trajectory-optimization_amd
A="DCOL_LIB=$L/lib_ab/libdcol.so"
CB="python3 tools/class_bench.py --small 0 --classes polytope-polytope,polytope-sphere,sphere-polytope,polytope-cone,cone-polytope,sphere-sphere,cone-cone,sphere-cone,capsule-sphere,capsule-cone,cylinder-sphere,cylinder-cone"
OUT=$O tools/gpu_session.sh "prod_a|300|$CB" "ilp_a|300|$A $CB" "prod_b|300|$CB" "ilp_b|300|$A $CB"
