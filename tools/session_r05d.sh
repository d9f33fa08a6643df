#!/bin/bash
# Round-5 session D: what a resident pair server costs a batch plan, per server knob.
O=gpurun_out/r05_d
mkdir -p $O
OUT=$O tools/gpu_session.sh \
  "tax_high|120|python3 tools/server_tax.py --label high" \
  "tax_normal|120|DCOL_PAIR_SERVER_PRIO=normal GPU_MAX_HW_QUEUES=8 python3 tools/server_tax.py --label normal_q8" \
  "tax_sleep100|120|DCOL_PAIR_SERVER_POLL_SLEEP=100 python3 tools/server_tax.py --label sleep100" \
  "tax_sleep10|120|DCOL_PAIR_SERVER_POLL_SLEEP=10 python3 tools/server_tax.py --label sleep10" \
  "bench_driver|300|python3 bench.py --gpus 1 --steps 20 --warmup 5"
