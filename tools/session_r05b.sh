#!/bin/bash
# Round-5 session B: LDS-rows build (lib_glds) against the round's baseline build
# (lib_r05base): bitwise outputs on the 1M mixed and 100k poly plans, then the per-class
# throughput of the one-lane x polytope classes (and controls), builds interleaved.
O=gpurun_out/r05_b
mkdir -p $O
L=dcol-trajectory-optimization_amd
C=cone-polytope,polytope-cone,capsule-polytope,polytope-capsule,cylinder-polytope,polytope-cylinder,polygon-polytope,polytope-polygon,sphere-polytope,polytope-polytope
OUT=$O tools/gpu_session.sh \
  "save_glds|300|DCOL_LIB=$L/lib_glds/libdcol.so python3 tools/lib_ab.py --save $O/glds.npz" \
  "save_base|300|DCOL_LIB=$L/lib_r05base/libdcol.so python3 tools/lib_ab.py --save $O/base.npz" \
  "compare|120|python3 tools/lib_ab.py --compare $O/glds.npz $O/base.npz" \
  "cls_glds1|300|DCOL_LIB=$L/lib_glds/libdcol.so python3 tools/class_bench.py --small 0 --classes $C" \
  "cls_base1|300|DCOL_LIB=$L/lib_r05base/libdcol.so python3 tools/class_bench.py --small 0 --classes $C" \
  "cls_glds2|300|DCOL_LIB=$L/lib_glds/libdcol.so python3 tools/class_bench.py --small 0 --classes $C" \
  "cls_base2|300|DCOL_LIB=$L/lib_r05base/libdcol.so python3 tools/class_bench.py --small 0 --classes $C"
rm -f $O/*.npz
