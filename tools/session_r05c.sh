#!/bin/bash
# Round-5 session C: server lifecycle / tax tests, the GPU suite, smoke, driver-length and
# default bench lines, rocprofv3 kernel trace + PMC passes of the headline workload.
O=gpurun_out/r05_c
mkdir -p $O
export TMPDIR=/tmp
B="python3 bench.py --no-cpu --no-altro --check 0 --steps 200 --warmup 100 --streams 1 --mixed-steps 0 --no-kernel-1m"
OUT=$O tools/gpu_session.sh \
  "newtests|400|python3 -u -m pytest tests/test_dropin.py -k 'process_exit or tax_batch' -v -s --timeout 300 --timeout-method thread" \
  "tests|900|python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread" \
  "smoke|120|python3 -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench_driver|300|python3 bench.py --gpus 1 --steps 20 --warmup 5" \
  "bench_default|400|python3 bench.py" \
  "trace|300|rocprofv3 --kernel-trace --stats -f csv -d $O/trace -o run -- $B" \
  "pmc_fetch|300|rocprofv3 --pmc FETCH_SIZE -f csv -d $O/pmc_fetch -o run -- $B" \
  "pmc_write|300|rocprofv3 --pmc WRITE_SIZE -f csv -d $O/pmc_write -o run -- $B"
