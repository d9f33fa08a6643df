#!/bin/bash
# GPU sessions of the build (one preset per gpurun call), run on the box through
#   gpurun -- tools/sessions.sh <preset> [outdir]
# each preset a list of "name|timeout_s|command" steps for tools/gpu_session.sh (each step
# under its own time limit; the session stops at the first fault-like exit).
P=${1:?preset}
O=gpurun_out/${2:-$P}
mkdir -p "$O"
export TMPDIR=/tmp
S=tools/gpu_session.sh
case $P in
  check)      # the round's closing check: GPU suite, smoke and the driver's command
    OUT=$O $S \
      "tests|900|python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread" \
      "smoke|120|python3 -c 'import __graft_entry__ as g; g.smoke()'" \
      "bench_driver|300|python3 bench.py --gpus 1 --steps 20 --warmup 5" ;;
  shards)     # configs[4]'s per-rank shards alone on one GPU, plan-policy A/B, kernel trace of 125k
    OUT=$O $S \
      "sweep|500|python3 tools/shard_bench.py --sweep --buckets" \
      "trace125k|200|rocprofv3 --kernel-trace -f csv -d $O/trace125k -o run -- python3 tools/shard_bench.py --worlds 8 --steps 20" ;;
  *) echo "unknown preset $P"; exit 2 ;;
esac
