#!/bin/bash
# Round-5 session W: the host-side cost of the headline's timed-region bracket (K = 20),
# with HIP's default 4 hardware queues and with bench.py's 8 (+ a torch side stream)
O=gpurun_out/r05_w
mkdir -p $O
OUT=$O tools/gpu_session.sh \
  "q4|200|K=20 R=15 python3 tools/bracket_probe.py" \
  "q8s|200|GPU_MAX_HW_QUEUES=8 EXTRA_STREAM=1 K=20 R=15 python3 tools/bracket_probe.py" \
  "q4s|200|EXTRA_STREAM=1 K=20 R=15 python3 tools/bracket_probe.py" \
  "q8|200|GPU_MAX_HW_QUEUES=8 K=20 R=15 python3 tools/bracket_probe.py" \
  "drv_q8|300|python3 bench.py --steps 20 --warmup 5 --no-cpu --no-altro" \
  "drv_q4|300|python3 bench.py --steps 20 --warmup 5 --no-cpu --no-altro --hw-queues 4"
