#!/bin/bash
# Round-5 final session: the round's build on a fresh box -- GPU suite, smoke, the default and
# driver-length lines, rocprofv3 kernel trace + PMC passes (FETCH_SIZE, WRITE_SIZE, FP64 mix,
# cycles) of the headline workload, the mixed workload's trace, the --gpus 8 gloo rehearsal.
NAME=${1:-r05_final}
O=gpurun_out/$NAME
mkdir -p $O
export TMPDIR=/tmp
B="python3 bench.py --no-cpu --no-altro --check 0 --steps 200 --warmup 100 --streams 1 --mixed-steps 0 --no-kernel-1m"
M="python3 bench.py --workload mixed1m --no-cpu --no-altro --check 0 --steps 20 --warmup 5"
OUT=$O tools/gpu_session.sh \
  "tests|900|python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread" \
  "smoke|120|python3 -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench_driver|300|python3 bench.py --gpus 1 --steps 20 --warmup 5" \
  "bench_default|400|python3 bench.py" \
  "trace|300|rocprofv3 --kernel-trace --stats -f csv -d $O/trace -o run -- $B" \
  "pmc_fetch|300|rocprofv3 --pmc FETCH_SIZE -f csv -d $O/pmc_fetch -o run -- $B" \
  "pmc_write|300|rocprofv3 --pmc WRITE_SIZE -f csv -d $O/pmc_write -o run -- $B" \
  "pmc_f64|300|rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 -f csv -d $O/pmc_f64 -o run -- $B" \
  "pmc_cycles|300|rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES -f csv -d $O/pmc_cycles -o run -- $B" \
  "trace_mixed|300|rocprofv3 --kernel-trace --stats -f csv -d $O/trace_mixed -o run -- $M" \
  "dp8_gloo|400|python3 bench.py --gpus 8 --backend gloo --no-cpu --steps 50 --warmup 10 --mixed-steps 5 --check 0"
