#!/bin/bash
# Round-5 session I: LDS rows for the cone x polygon bucket (lib) against the BOX build
# without them (lib_r05base), per class, interleaved; the outputs bitwise.
O=gpurun_out/r05_i
mkdir -p $O
L=dcol-trajectory-optimization_amd
C=cone-polygon,polygon-cone,polytope-polytope,cone-polytope,polytope-cone
OUT=$O tools/gpu_session.sh \
  "save_new|300|python3 tools/lib_ab.py --save $O/new.npz" \
  "save_base|300|DCOL_LIB=$L/lib_r05base/libdcol.so python3 tools/lib_ab.py --save $O/base.npz" \
  "compare|120|python3 tools/lib_ab.py --compare $O/new.npz $O/base.npz" \
  "cls_new1|300|python3 tools/class_bench.py --small 0 --classes $C" \
  "cls_base1|300|DCOL_LIB=$L/lib_r05base/libdcol.so python3 tools/class_bench.py --small 0 --classes $C" \
  "cls_new2|300|python3 tools/class_bench.py --small 0 --classes $C" \
  "cls_base2|300|DCOL_LIB=$L/lib_r05base/libdcol.so python3 tools/class_bench.py --small 0 --classes $C"
rm -f $O/*.npz
