#!/bin/bash
# Round-5 session AF: machine schedule per unit -- all 27 classes with the product library and
# its twin (every unit under the other scheduling strategy, register G rows), interleaved
O=gpurun_out/r05_af
mkdir -p $O
L=dcol-trajectory-optimization_amd
X="DCOL_LIB=$L/lib_xcheck/libdcol.so"
CB="python3 tools/class_bench.py --small 0"
OUT=$O tools/gpu_session.sh "prod_a|400|$CB" "twin_a|400|$X $CB" "prod_b|400|$CB" "twin_b|400|$X $CB"
