#!/bin/bash
# Round-5 session L: sphere x box at one lane per pair with LDS rows (lib) against the LPP-2
# kernel (lib_r05base); the GPU suite (the 1M mixed set against the C oracle); driver bench.
O=gpurun_out/r05_l
mkdir -p $O
L=dcol-trajectory-optimization_amd
C=sphere-polytope,polytope-sphere,cone-polytope,polytope-polytope
OUT=$O tools/gpu_session.sh \
  "cls_new1|300|python3 tools/class_bench.py --small 1000 --classes $C" \
  "cls_base1|300|DCOL_LIB=$L/lib_r05base/libdcol.so python3 tools/class_bench.py --small 1000 --classes $C" \
  "cls_new2|300|python3 tools/class_bench.py --small 1000 --classes $C" \
  "cls_base2|300|DCOL_LIB=$L/lib_r05base/libdcol.so python3 tools/class_bench.py --small 1000 --classes $C" \
  "tests|900|python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread" \
  "bench_driver|300|python3 bench.py --gpus 1 --steps 20 --warmup 5"
