#!/bin/bash
# Round-5 session T: fan-out width of the 1M mixed plan (DCOL_SIDE_STREAMS 1 / 2 / 3),
# synchronised steps, then the bench's mixed1m line at 2 and 3 side streams; a kernel trace
# of the 2-side-stream step.
O=gpurun_out/r05_t
mkdir -p $O
M="python3 tools/mixed_buckets.py --steps 60"
B="python3 bench.py --workload mixed1m --no-cpu --steps 20 --warmup 5"
OUT=$O tools/gpu_session.sh \
  "s1_a|200|DCOL_SIDE_STREAMS=1 $M" "s2_a|200|DCOL_SIDE_STREAMS=2 $M" "s3_a|200|$M" \
  "s1_b|200|DCOL_SIDE_STREAMS=1 $M" "s2_b|200|DCOL_SIDE_STREAMS=2 $M" "s3_b|200|$M" \
  "bench_s2_a|300|DCOL_SIDE_STREAMS=2 $B" "bench_s3_a|300|$B" \
  "bench_s2_b|300|DCOL_SIDE_STREAMS=2 $B" "bench_s3_b|300|$B" \
  "trace_s2|300|DCOL_SIDE_STREAMS=2 rocprofv3 --kernel-trace -f csv -d $O/trace_s2 -o run -- $M"
