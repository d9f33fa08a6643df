#!/bin/bash
# Round-5 session O: the LPP-1 BOX copy with LDS rows at two waves per SIMD (DCOL_LPP=1)
# against the LPP-2 three-wave BOX kernel: parity vs the C oracle, then interleaved headline
# serial / pipelined rates and the 1M kernel-only rate.
O=gpurun_out/r05_o
mkdir -p $O
B="python3 bench.py --no-cpu --no-altro --mixed-steps 0 --check 0"
T="python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fullsize.py -k"
OUT=$O tools/gpu_session.sh \
  "par1|400|DCOL_LPP=1 $T 'whole_batch or chunked or swap'" \
  "l1_a|200|DCOL_LPP=1 $B --steps 20 --warmup 5" \
  "l2_a|200|$B --steps 20 --warmup 5" \
  "l1_b|200|DCOL_LPP=1 $B --steps 200 --warmup 20" \
  "l2_b|200|$B --steps 200 --warmup 20" \
  "l1_c|200|DCOL_LPP=1 $B --steps 20 --warmup 5" \
  "l2_c|200|$B --steps 20 --warmup 5"
