#!/usr/bin/env python3
"""Summarise a rocprofv3 PMC pass of the headline solve kernel (SQ_INSTS_VALU,
SQ_INSTS_VALU_{ADD,MUL,FMA,TRANS}_F64, GRBM_GUI_ACTIVE in one pass) into
profiles/pmc_fp64.json -- the EXECUTED FP64 work per launch that bench.py puts beside the
counted-flop roofline (roofline_fp64.executed_*):
  executed flops / launch = (ADD + MUL + 2 FMA + TRANS) F64 wave-instructions x 64 lanes
  VALU issue fraction     = SQ_INSTS_VALU x 4 cycles (a wave64 VALU instruction on a 16-lane
                            SIMD) / (SIMDs x GRBM_GUI_ACTIVE / 8)  (GRBM: the sum over the
                            8 XCDs, MI355X_MICROARCH.md "DVFS give-back")
  FP64 share of VALU      = F64 instructions / SQ_INSTS_VALU
Medians over the kernel's dispatches.
Usage: tools/pmc_fp64.py run_counter_collection.csv OUT.json [pairs_per_launch] [kernel_substr]"""
import csv
import json
import statistics
import sys

SIMDS = 1024   # MI355X: 256 CUs x 4 SIMDs


def main():
    path, out = sys.argv[1], sys.argv[2]
    pairs = int(sys.argv[3]) if len(sys.argv) > 3 else 100_000
    ksub = sys.argv[4] if len(sys.argv) > 4 else "prox_kernel<4, 0, 12, 2, 3, "   # the BOX kernel (FD-only copy: FL 73)
    vals, name = {}, None
    for r in csv.DictReader(open(path)):
        if ksub in r["Kernel_Name"]:
            name = r["Kernel_Name"]
            vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    med = {k: statistics.median(v) for k, v in vals.items()}
    f64 = {k: med.get(f"SQ_INSTS_VALU_{k}_F64", 0.0) for k in ("ADD", "MUL", "FMA", "TRANS")}
    flops = 64.0 * (f64["ADD"] + f64["MUL"] + 2.0 * f64["FMA"] + f64["TRANS"])
    valu = med["SQ_INSTS_VALU"]
    cycles = med["GRBM_GUI_ACTIVE"] / 8.0
    d = {"kernel": name, "dispatches": min(len(v) for v in vals.values()), "pairs_per_launch": pairs,
         "counters_median": med,
         "executed_flops_per_launch": flops, "executed_flops_per_pair": flops / pairs,
         "fp64_instructions_per_launch": sum(f64.values()), "valu_instructions_per_launch": valu,
         "fp64_share_of_valu": sum(f64.values()) / valu,
         "valu_issue_frac": valu * 4.0 / (SIMDS * cycles),
         "note": "executed = (ADD + MUL + 2 FMA + TRANS) F64 wave-instructions x 64; VALU issue = SQ_INSTS_VALU x 4 "
                 "/ (1024 SIMDs x GRBM_GUI_ACTIVE / 8) over the kernel's active cycles in the PMC run"}
    json.dump(d, open(out, "w"), indent=1)
    print(json.dumps(d))


if __name__ == "__main__":
    main()
