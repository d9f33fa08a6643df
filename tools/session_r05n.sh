#!/bin/bash
# Round-5 session N: GPU suite on the current build, all 27 classes, the mixed workload's
# kernel trace.
O=gpurun_out/r05_n
mkdir -p $O
export TMPDIR=/tmp
M="python3 bench.py --workload mixed1m --no-cpu --no-altro --check 0 --steps 20 --warmup 5"
OUT=$O tools/gpu_session.sh \
  "tests|900|python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread" \
  "cls|400|python3 tools/class_bench.py --small 0" \
  "trace_mixed|300|rocprofv3 --kernel-trace --stats -f csv -d $O/trace_mixed -o run -- $M"
