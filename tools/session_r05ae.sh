#!/bin/bash
# Round-5 session AE: per-class throughput of the round's build (all 27 classes) and PMC
# passes over the 1M mixed plan (FP64 instruction mix, wave cycles) per kernel
O=gpurun_out/r05_ae
mkdir -p $O
export TMPDIR=/tmp
M="python3 tools/mixed_buckets.py --steps 5"
OUT=$O tools/gpu_session.sh \
  "cls_all27|400|python3 tools/class_bench.py" \
  "pmc_f64|120|timeout -s KILL 100 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 -f csv -d $O/pmc_f64 -o run -- $M" \
  "pmc_cyc|120|timeout -s KILL 100 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES -f csv -d $O/pmc_cyc -o run -- $M"
