#!/bin/bash
# Build lib/libdcol.so variants with different compiler options into lib_sweep/<name>/ for
# A/B runs on the GPU box (bench.py picks one with DCOL_LIB=...).  Host-side only.
#   tools/flag_sweep.sh name "extra flags" [name "flags"] ...
set -e
cd "$(dirname "$0")/../dcol-trajectory-optimization_amd/csrc"
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  out=../../lib_sweep/$name
  mkdir -p "$out"
  make -s -j8 OUTDIR="$out" BUILD="build_sweep/$name" EXTRA="$flags" "$out/libdcol.so"
  echo "built $name: $flags"
done
