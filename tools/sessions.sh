#!/bin/bash
# GPU sessions of the build (one preset per gpurun call), run on the box through
#   gpurun -- tools/sessions.sh <preset> [outdir]
# each preset a list of "name|timeout_s|command" steps for tools/gpu_session.sh (each step
# under its own time limit; the session stops at the first fault-like exit).  Replaces the
# per-session scripts of rounds 1-5 (tools/session_r05*.sh, profile_session.sh: their logs
# under profiles/ name the commands they ran).
P=${1:?preset}
O=gpurun_out/${2:-$P}
mkdir -p "$O"
export TMPDIR=/tmp
S=tools/gpu_session.sh
# the headline kernel alone (configs[3], one stream) for PMC passes, and the FP64 counter set
HB="python3 bench.py --no-cpu --no-altro --check 0 --steps 200 --warmup 100 --streams 1 --mixed-steps 0 --no-kernel-1m"
F64="SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 GRBM_GUI_ACTIVE"
M="python3 bench.py --workload mixed1m --no-cpu --no-altro --check 0 --steps 20 --warmup 5"
case $P in
  final)      # a full measurement session for profiles/<outdir>/: GPU suite, smoke, the default
              # line and the driver's command, kernel traces of the headline and the mixed
              # step, the PMC passes of the headline kernel (one counter group per pass), the
              # eight-rank gloo rehearsal of --gpus 8
    OUT=$O $S \
      "tests|900|python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread" \
      "smoke|120|python3 -c 'import __graft_entry__ as g; g.smoke()'" \
      "bench_default|500|python3 bench.py" \
      "bench_driver|300|python3 bench.py --gpus 1 --steps 20 --warmup 5" \
      "trace|300|rocprofv3 --kernel-trace --stats -f csv -d $O/trace -o run -- $HB" \
      "trace_mixed|300|rocprofv3 --kernel-trace --stats -f csv -d $O/trace_mixed -o run -- $M" \
      "pmc_fetch|150|timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d $O/pmc_fetch -o run -- $HB" \
      "pmc_write|150|timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d $O/pmc_write -o run -- $HB" \
      "pmc_f64|150|timeout -s KILL 120 rocprofv3 --pmc $F64 -f csv -d $O/pmc_f64 -o run -- $HB" \
      "pmc_cycles|150|timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES -f csv -d $O/pmc_cycles -o run -- $HB" \
      "dp8_gloo|400|python3 bench.py --gpus 8 --backend gloo --no-cpu --steps 50 --warmup 10 --mixed-steps 5 --check 0" ;;
  classes)    # all 27 mixed classes, 200k pairs each (tools/class_bench.py)
    OUT=$O $S "cls_all27|500|python3 tools/class_bench.py" ;;
  mixed)      # the 1M mixed plan's buckets and a kernel trace of synchronised steps; per-kernel PMC
    OUT=$O $S \
      "buckets|200|python3 tools/mixed_buckets.py --steps 30" \
      "trace|300|rocprofv3 --kernel-trace -f csv -d $O/trace -o run -- python3 tools/mixed_buckets.py --steps 30" \
      "pmc_f64|150|timeout -s KILL 120 rocprofv3 --pmc $F64 -f csv -d $O/pmc_f64 -o run -- python3 tools/mixed_buckets.py --steps 5" \
      "pmc_cyc|150|timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES -f csv -d $O/pmc_cyc -o run -- python3 tools/mixed_buckets.py --steps 5" ;;
  dropin)     # the drop-in's per-call latency (quadrotor hallway sweeps)
    OUT=$O $S "dropin|300|python3 tools/dropin_ab.py --rounds 2" ;;
  check)      # the round's closing check: GPU suite, smoke and the driver's command
    OUT=$O $S \
      "tests|900|python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread" \
      "smoke|120|python3 -c 'import __graft_entry__ as g; g.smoke()'" \
      "bench_driver|300|python3 bench.py --gpus 1 --steps 20 --warmup 5" ;;
  shards)     # configs[4]'s per-rank shards alone on one GPU, plan-policy A/B, kernel trace of 125k
    OUT=$O $S \
      "sweep|600|python3 tools/shard_bench.py --sweep --buckets --only=$ONLY" \
      "trace125k|200|rocprofv3 --kernel-trace -f csv -d $O/trace125k -o run -- python3 tools/shard_bench.py --worlds 8 --steps 20" ;;
  shards2)    # the small-plan / fused policies for the 125k-250k shards; trace of the fused 125k; FP64 PMC
    OUT=$O ONLY=default,small_fused,small_fused_keyorder,small_nofuse,lat_per_launch $S \
      "sweep|600|python3 tools/shard_bench.py --sweep --buckets --only=default,small_fused,small_fused_keyorder,small_nofuse,lat_per_launch" \
      "trace125k_fused|200|DCOL_SMALL_PLAN_LANES=500000 rocprofv3 --kernel-trace -f csv -d $O/trace125k_fused -o run -- python3 tools/shard_bench.py --worlds 8 --steps 20" \
      "pmc_f64|150|timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 GRBM_GUI_ACTIVE -f csv -d $O/pmc_f64 -o run -- python3 bench.py --no-cpu --no-altro --check 0 --steps 200 --warmup 100 --streams 1 --mixed-steps 0 --no-kernel-1m" ;;
  shards3)    # the packed launch by threshold, shard sizes 1M / N for N = 1 .. 32
    W=1,2,3,4,6,8,12,16,32
    OUT=$O $S \
      "sweep|700|python3 tools/shard_bench.py --sweep --worlds $W --only=default,pack_off,pack_1m,pack_all,pack_keyorder" \
      "trace125k_packed|200|rocprofv3 --kernel-trace -f csv -d $O/trace125k_packed -o run -- python3 tools/shard_bench.py --worlds 8 --steps 20" \
      "bench|400|python3 bench.py --no-cpu --no-altro --steps 200 --warmup 50" \
      "pmc_fetch|150|timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d $O/pmc_fetch -o run -- $HB" \
      "pmc_write|150|timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d $O/pmc_write -o run -- $HB" \
      "pmc_f64|150|timeout -s KILL 120 rocprofv3 --pmc $F64 -f csv -d $O/pmc_f64 -o run -- $HB" ;;
  shards4)    # the round-6 plan policy (packed mid-size plans, packed unfused small plans) against
              # the fan-out, shard sizes 1M / N for N = 1 .. 128; then the whole GPU suite
    W=1,2,4,8,16,32,64,128
    OUT=$O $S \
      "sweep|700|python3 tools/shard_bench.py --sweep --worlds $W --only=default,pack_off,small_fanout" \
      "tests|1000|python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread" ;;
  tests)      # the GPU suite (or the tests named by $K, a pytest -k expression)
    OUT=$O $S "tests|1000|python3 -u -m pytest tests -m gpu -q -s --timeout 300 --timeout-method thread ${K:+-k \"$K\"}" ;;
  quick)      # tests named by $K, then a short bench line (every section but the CPU baselines)
    OUT=$O $S "tests|900|python3 -u -m pytest tests -m gpu -q -s --timeout 300 --timeout-method thread -k \"$K\"" \
      "bench|400|python3 bench.py --no-cpu --steps 100 --warmup 20" ;;
  shards5)    # the two-family packed launch by threshold; tests named by $K
    W=1,2,3,4,6,8,16,32,64,128,512,4096
    OUT=$O $S \
      "sweep|700|python3 tools/shard_bench.py --sweep --worlds $W --only=default,pack_all,pack_off" \
      "trace125k|200|rocprofv3 --kernel-trace -f csv -d $O/trace125k -o run -- python3 tools/shard_bench.py --worlds 8 --steps 20" \
      "tests|900|python3 -u -m pytest tests -m gpu -q -s --timeout 300 --timeout-method thread -k \"$K\"" ;;
  split)      # the split-SOC copies (DCOL_SPLIT=1, Solver SPLIT) of {capsule, cylinder} x polytope:
              # parity (env-variant test) and per-class time against the default (LPP 1) and the
              # two-lane copies without the split (DCOL_LPP=2)
    C=capsule-polytope,polytope-capsule,cylinder-polytope,polytope-cylinder
    CB="python3 tools/class_bench.py --small 0 --reps 20 --classes $C"
    OUT=$O $S \
      "tests|600|python3 -u -m pytest tests -m gpu -q -s --timeout 300 --timeout-method thread -k env_variants" \
      "cls_default|300|$CB" \
      "cls_split|300|DCOL_SPLIT=1 $CB" \
      "cls_split_w2|300|DCOL_SPLIT=1 DCOL_WPS=2 $CB" \
      "cls_lpp2|300|DCOL_LPP=2 $CB" \
      "cls_default2|300|$CB" ;;
  *) echo "unknown preset $P"; exit 2 ;;
esac
