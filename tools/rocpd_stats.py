#!/usr/bin/env python3
"""Kernel statistics from a rocprofv3 SQLite result (run_results.db) -> CSV on stdout
(same columns as rocprofv3's kernel_stats.csv: Name, Calls, TotalDurationNs,
AverageNs, Percentage, MinNs, MaxNs).  Usage: tools/rocpd_stats.py gpurun_out/x/run_results.db"""
import sqlite3
import sys


def main(path):
    db = sqlite3.connect(path)
    rows = db.execute("select name, count(*), sum(end - start), avg(end - start), min(end - start), max(end - start) "
                      "from kernels group by name order by sum(end - start) desc").fetchall()
    total = sum(r[2] for r in rows) or 1
    print('"Name","Calls","TotalDurationNs","AverageNs","Percentage","MinNs","MaxNs"')
    for name, n, tot, avg, mn, mx in rows:
        print(f'"{name}",{n},{tot},{avg:.1f},{100.0 * tot / total:.3f},{mn},{mx}')


if __name__ == "__main__":
    main(sys.argv[1])
