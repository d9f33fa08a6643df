#!/bin/bash
# Round-5 session F: pair server giving way to batch launches; exit-path tests; GPU suite.
O=gpurun_out/r05_f
mkdir -p $O
OUT=$O tools/gpu_session.sh \
  "tax_yield|120|python3 tools/server_tax.py --label cumask_yield" \
  "tax_noyield|120|DCOL_PAIR_SERVER_YIELD=0 python3 tools/server_tax.py --label cumask_noyield" \
  "tax_noyield_q8|120|DCOL_PAIR_SERVER_YIELD=0 GPU_MAX_HW_QUEUES=8 python3 tools/server_tax.py --label cumask_noyield_q8" \
  "newtests|400|python3 -u -m pytest tests/test_dropin.py -k 'process_exit or gives_way' -v -s --timeout 300 --timeout-method thread" \
  "tests|900|python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread" \
  "bench_driver|300|python3 bench.py --gpus 1 --steps 20 --warmup 5"
