#!/usr/bin/env python3
"""Per-step timeline of a multi-bucket plan from a rocprofv3 kernel trace
(run_kernel_trace.csv): the solve kernels of each step with their stream, start and end
relative to the step's first kernel, and per variant the median duration over the steps.
  python3 tools/mixed_timeline.py <run_kernel_trace.csv> [steps to print]"""
import csv
import re
import statistics
import sys


def steps_of(path):
    rows = [r for r in csv.DictReader(open(path)) if "prox_kernel" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Correlation_Id"]))   # issue order: a step's launches are consecutive
    per = {}
    for r in rows:   # launches per step = distinct variants (each bucket launches once per step)
        per.setdefault(r["Kernel_Name"], 0)
    k = len(per)
    # a step = k consecutive launches in issue order
    out, cur = [], []
    for r in rows:
        if len(cur) == k:
            out.append(cur)
            cur = []
        cur.append(r)
    if len(cur) == k:
        out.append(cur)
    return out


def name(r):
    return re.search(r"prox_kernel<([^>]*)>", r["Kernel_Name"]).group(1).replace(" ", "")


def main():
    path = sys.argv[1]
    show = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    st = steps_of(path)
    dur, spans = {}, []
    for s in st:
        t0 = min(int(r["Start_Timestamp"]) for r in s)
        t1 = max(int(r["End_Timestamp"]) for r in s)
        spans.append((t1 - t0) / 1e3)
        for r in s:
            dur.setdefault(name(r), []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print(f"steps {len(st)}  span us median {statistics.median(spans):.1f}  min {min(spans):.1f}  max {max(spans):.1f}")
    tot = 0.0
    for k, v in sorted(dur.items(), key=lambda kv: -statistics.median(kv[1])):
        m = statistics.median(v)
        tot += m
        print(f"  {k:24s} median {m:7.1f} us  min {min(v):7.1f}  max {max(v):7.1f}")
    print(f"  sum of medians {tot:.1f} us")
    for s in st[len(st) // 2:len(st) // 2 + show]:
        t0 = min(int(r["Start_Timestamp"]) for r in s)
        print("step")
        for r in s:
            print(f"  s{r['Stream_Id']:>3} {name(r):24s} {(int(r['Start_Timestamp']) - t0) / 1e3:7.1f} "
                  f"{(int(r['End_Timestamp']) - t0) / 1e3:7.1f}")


if __name__ == "__main__":
    main()
