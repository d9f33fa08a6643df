#!/usr/bin/env python3
"""Per-launch durations of the solve kernel in a rocprofv3 kernel trace, in launch order,
with the idle gaps between launches -- the clock ramp under sustained load (DESIGN.md
section 3, "Short driver runs measure the clock ramp").

  tools/clock_ramp.py profiles/r02_v9/trace/run_kernel_trace.csv [kernel-substring]
"""
import csv
import sys


def main():
    path = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else "prox_kernel"
    rows = [r for r in csv.DictReader(open(path)) if sub in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
    gap = [0.0] + [(int(rows[i]["Start_Timestamp"]) - int(rows[i - 1]["End_Timestamp"])) / 1e3
                   for i in range(1, len(rows))]
    print(f"{len(rows)} launches of *{sub}*; duration in us per block of 20 launches "
          "(mean), and the largest idle gap before the block")
    for i in range(0, len(dur), 20):
        d = dur[i:i + 20]
        print(f"{i:5d}  {sum(d) / len(d):7.1f} us   gap {max(gap[i:i + 20]):9.1f} us")


if __name__ == "__main__":
    main()
