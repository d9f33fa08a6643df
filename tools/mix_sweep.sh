for lib in lib_sweep/*/libdcol.so; do
  name=$(basename "$(dirname "$lib")")
  DCOL_LIB=$PWD/$lib timeout -k 10 200 python3 bench.py --workload mixed1m --steps 5 --warmup 2 --check 64 > gpurun_out/mix_$name.log 2>&1 || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/mix_$name.log').read().strip().splitlines()[-1]);print('$name', round(d['value']/1e8,3), round(d['ms_per_step'],3), d['parity_check'])"
  DCOL_LIB=$PWD/$lib timeout -k 10 200 python3 tools/altro_rep.py quadrotor coneThroughWall || exit 1
done
