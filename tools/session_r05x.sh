#!/bin/bash
# Round-5 session X: the headline batch with its last partial round split off to a second stream
O=gpurun_out/r05_x
mkdir -p $O
OUT=$O tools/gpu_session.sh "split|200|python3 tools/tail_split_probe.py 100"
