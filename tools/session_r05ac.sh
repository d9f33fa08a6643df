#!/bin/bash
# Round-5 session AC: the timed regions' end waits as a spin on the end event (default) against
# the blocking wait (DCOL_BENCH_SPIN=0), the driver's command, interleaved
O=gpurun_out/r05_ac
mkdir -p $O
B="python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-altro"
OUT=$O tools/gpu_session.sh "spin_a|200|$B" "block_a|200|DCOL_BENCH_SPIN=0 $B" "spin_b|200|$B" "block_b|200|DCOL_BENCH_SPIN=0 $B" \
  "spin_c|200|$B" "block_c|200|DCOL_BENCH_SPIN=0 $B" "spin_d|200|$B" "block_d|200|DCOL_BENCH_SPIN=0 $B"
