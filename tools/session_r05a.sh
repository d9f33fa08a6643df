#!/bin/bash
# Round-5 session A: the new server-lifecycle / batch-tax tests, the GPU suite, smoke, the
# default and driver-length bench lines, the eight-rank gloo rehearsal of --gpus 8.
OUT=gpurun_out/r05_a tools/gpu_session.sh \
  "newtests|400|python3 -u -m pytest tests/test_dropin.py -k 'process_exit or tax_batch' -v -s --timeout 300 --timeout-method thread" \
  "tests|900|python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread" \
  "smoke|120|python3 -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench_default|400|python3 bench.py" \
  "bench_driver|300|python3 bench.py --gpus 1 --steps 20 --warmup 5" \
  "dp8_gloo|400|python3 bench.py --gpus 8 --backend gloo --no-cpu --steps 50 --warmup 10 --mixed-steps 5 --check 0"
