#!/bin/bash
# Round-5 session Q: BOX kernel at four waves per SIMD with LDS rows (lib_ab, WPS 14: 128
# VGPRs, 24 scratch instructions per loop) against the three-wave register-rows kernel (lib):
# parity of the A copy vs the C oracle, then interleaved 100k / 98,304 / 1M rates.
O=gpurun_out/r05_q
mkdir -p $O
L=dcol-trajectory-optimization_amd
A="DCOL_LIB=$L/lib_ab/libdcol.so"
B="python3 bench.py --no-cpu --no-altro --mixed-steps 0 --check 0 --steps 50 --warmup 10"
T="python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fullsize.py -k"
OUT=$O tools/gpu_session.sh \
  "par4|400|$A $T 'whole_batch or chunked or swap'" \
  "w4_a|200|$A $B" "w3_a|200|$B" \
  "w4_n98|200|$A $B --pairs 98304 --no-kernel-1m" "w3_n98|200|$B --pairs 98304 --no-kernel-1m" \
  "w4_b|200|$A $B" "w3_b|200|$B" \
  "w4_n131|200|$A $B --pairs 131072 --no-kernel-1m" "w3_n131|200|$B --pairs 131072 --no-kernel-1m"
