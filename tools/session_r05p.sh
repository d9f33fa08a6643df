#!/bin/bash
# Round-5 session P: the BOX kernel's launch-size curve around the 100k batch (waves of 32
# pairs over 3,072 three-wave slots) and its iteration-cap curve: where the 100k launch's
# time above the 1M rate goes.
O=gpurun_out/r05_p
mkdir -p $O
B="python3 bench.py --no-cpu --no-altro --mixed-steps 0 --check 0 --no-kernel-1m --steps 50 --warmup 10"
specs=()
for n in 24576 49152 73728 98304 100000 101376 122880 147456 196608 294912; do specs+=("n$n|120|$B --pairs $n"); done
for c in 6 8 9 10 11 12 13; do specs+=("cap$c|120|$B --max-iter $c"); done
OUT=$O tools/gpu_session.sh "${specs[@]}"
