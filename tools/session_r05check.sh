#!/bin/bash
# Round-5 closing check: GPU suite, smoke and the driver's command on the tree as committed
O=gpurun_out/${1:-r05_check}
mkdir -p $O
OUT=$O tools/gpu_session.sh \
  "tests|900|python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread" \
  "smoke|120|python3 -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench_driver|300|python3 bench.py --gpus 1 --steps 20 --warmup 5"
