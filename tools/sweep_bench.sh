#!/bin/bash
# On the GPU box: bench every lib_sweep/<name>/libdcol.so (100k and 1M pairs), one line each.
#   tools/sweep_bench.sh [extra bench.py args]
mkdir -p gpurun_out/sweep
for lib in lib_sweep/*/libdcol.so; do
  name=$(basename "$(dirname "$lib")")
  for n in 100000 1000000; do
    DCOL_LIB=$PWD/$lib timeout -k 10 120 python3 bench.py --no-cpu --no-altro --check 64 --pairs $n "$@" \
      > gpurun_out/sweep/$name.$n.log 2>&1 || { echo "$name $n FAILED rc=$?"; exit 1; }
    python3 -c "import json;d=json.loads(open('gpurun_out/sweep/$name.$n.log').read().strip().splitlines()[-1]);print('$name', $n, round(d['value']/1e8,3), round(d['kernel_ms'],4), d.get('parity_check',{}).get('grad_ok'))"
  done
done
