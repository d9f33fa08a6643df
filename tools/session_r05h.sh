#!/bin/bash
# Round-5 session H: the BOX (axis-pair) box x box kernel: GPU suite (100k / 1M oracle
# comparisons), driver-length and default bench lines, rocprofv3 trace of the headline.
O=gpurun_out/r05_h
mkdir -p $O
export TMPDIR=/tmp
B="python3 bench.py --no-cpu --no-altro --check 0 --steps 200 --warmup 100 --streams 1 --mixed-steps 0 --no-kernel-1m"
OUT=$O tools/gpu_session.sh \
  "fullsize|600|python3 -u -m pytest tests/test_gpu_fullsize.py tests/test_plan_buckets.py -v --timeout 300 --timeout-method thread" \
  "tests|900|python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread" \
  "bench_driver|300|python3 bench.py --gpus 1 --steps 20 --warmup 5" \
  "bench_default|400|python3 bench.py" \
  "trace|300|rocprofv3 --kernel-trace --stats -f csv -d $O/trace -o run -- $B"
