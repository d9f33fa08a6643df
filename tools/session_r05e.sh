#!/bin/bash
# Round-5 session E: the pair server on a CU-masked stream: batch tax and queue sharing
# against the normal / high-priority alternatives (GPU_MAX_HW_QUEUES at HIP's default 4).
O=gpurun_out/r05_e
mkdir -p $O
OUT=$O tools/gpu_session.sh \
  "tax_cumask|120|python3 tools/server_tax.py --label cumask" \
  "tax_normal|120|DCOL_PAIR_SERVER_STREAM=normal python3 tools/server_tax.py --label normal" \
  "tax_high|120|DCOL_PAIR_SERVER_STREAM=high python3 tools/server_tax.py --label high" \
  "tax_cumask2|120|python3 tools/server_tax.py --label cumask2"
