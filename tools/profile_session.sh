#!/bin/bash
# Full measurement session on the GPU box for profiles/<name>/ (run through gpurun):
#   GPU parity tests, the default bench line, a kernel-trace/stats pass and separate PMC
#   passes (FETCH_SIZE, WRITE_SIZE, FP64 instruction mix, SQ cycles) of the bench workload.
#   tools/profile_session.sh <name>
set -o pipefail
NAME=${1:?name}
OUT=gpurun_out/$NAME
mkdir -p "$OUT"
export TMPDIR=/tmp
B="python3 bench.py --no-cpu --no-altro --check 0 --steps 200 --warmup 100 --streams 1 --mixed-steps 0 --no-kernel-1m"
M="python3 bench.py --workload mixed1m --no-cpu --no-altro --check 0 --steps 20 --warmup 5"
OUT=$OUT tools/gpu_session.sh \
  "tests|600|python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread" \
  "smoke|120|python3 -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench_default|400|python3 bench.py" \
  "bench_driver|400|python3 bench.py --gpus 1 --steps 20 --warmup 5" \
  "trace|300|rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- $B" \
  "trace_mixed|300|rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace_mixed -o run -- $M" \
  "pmc_fetch|300|rocprofv3 --pmc FETCH_SIZE -f csv -d $OUT/pmc_fetch -o run -- $B" \
  "pmc_write|300|rocprofv3 --pmc WRITE_SIZE -f csv -d $OUT/pmc_write -o run -- $B" \
  "pmc_f64|300|rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 -f csv -d $OUT/pmc_f64 -o run -- $B" \
  "pmc_cycles|300|rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES -f csv -d $OUT/pmc_cycles -o run -- $B"
