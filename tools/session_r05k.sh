#!/bin/bash
# Round-5 session K: the shader clock during the drop-in sweeps (rocm-smi, read-only, every
# ~0.3 s beside the stamps tool), the default poll against a poll without s_sleep.
O=gpurun_out/r05_k
mkdir -p $O
L=dcol-trajectory-optimization_amd/lib_stamps/libdcol.so
clk() { for i in $(seq 60); do date +%s.%N; rocm-smi --showclocks 2>&1 | grep -i "sclk\|fclk\|mclk"; sleep 0.2; done > $O/$1 2>&1; }
clk clk_idle.log
clk clk_default.log & P=$!
timeout -k 10 120 env DCOL_LIB=$L python3 tools/dropin_stamps.py --label default --sweeps 4 > $O/stamps_default.log 2>&1; r1=$?
wait $P
clk clk_nosleep.log & P=$!
timeout -k 10 120 env DCOL_LIB=$L DCOL_PAIR_SERVER_POLL_SLEEP=-1 python3 tools/dropin_stamps.py --label nosleep --sweeps 4 > $O/stamps_nosleep.log 2>&1; r2=$?
wait $P
echo "rc $r1 $r2"
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r05_k/bench_driver.log 2>&1
