#!/bin/bash
# Round-5 session M: BOX kernel at three waves per SIMD (lib) against two (lib_r05base):
# headline serial rate, kernel time, 1M kernel-only rate; interleaved.
O=gpurun_out/r05_m
mkdir -p $O
L=dcol-trajectory-optimization_amd
B="python3 bench.py --no-cpu --no-altro --mixed-steps 0 --check 0"
OUT=$O tools/gpu_session.sh \
  "w3_a|200|$B --steps 20 --warmup 5" \
  "w2_a|200|DCOL_LIB=$L/lib_r05base/libdcol.so $B --steps 20 --warmup 5" \
  "w3_b|200|$B --steps 200 --warmup 20" \
  "w2_b|200|DCOL_LIB=$L/lib_r05base/libdcol.so $B --steps 200 --warmup 20" \
  "w3_c|200|$B --steps 20 --warmup 5" \
  "w2_c|200|DCOL_LIB=$L/lib_r05base/libdcol.so $B --steps 20 --warmup 5"
