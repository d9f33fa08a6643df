#!/bin/bash
# Per-kernel VGPRs / scratch / occupancy of one kernel TU (default N=4):  tools/kres.sh [n]
N=${1:-4}
cd "$(dirname "$0")/../dcol-trajectory-optimization_amd/csrc" || exit 1
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -c dcol_kernels_n$N.hip -o /dev/null \
    -Rpass-analysis=kernel-resource-usage 2>&1 | python3 -c '
import re, sys
name = None
for ln in sys.stdin:
    m = re.search(r"Function Name: (\S+)", ln)
    if m:
        name = re.sub(r"_ZN4dcol11prox_kernelILi(\d)ELi(\d)ELi(\d+)ELi(\d)ELi(\d)ELb(\d)EEEvNS_5KArgsE", r"<\1,\2,\3,\4,\5,\6>", m.group(1)); continue
    for key in ("VGPRs", "AGPRs", "ScratchSize \\[bytes/lane\\]", "Occupancy \\[waves/SIMD\\]"):
        m = re.search(key + r": (\d+)", ln)
        if m: print(name, key.split()[0], m.group(1))
' | paste -d" " - - - - | awk '{print $1, "vgpr", $3, "agpr", $6, "scratch", $9, "occ", $12}'
