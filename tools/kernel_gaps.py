#!/usr/bin/env python3
"""Gaps between consecutive kernels of one step call, from a rocprofv3
--kernel-trace CSV (kernel_trace.csv): for every pair of back-to-back
launches whose names contain the given string (default mh_step), the
time from one's end to the next one's start, and the kernels' own durations.
Usage: kernel_gaps.py <kernel_trace.csv> [prefix]
"""
import csv
import sys

import numpy as np

if __name__ == "__main__":
    path = sys.argv[1]
    prefix = sys.argv[2] if len(sys.argv) > 2 else "mh_step"
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    gaps, durs = {}, {}
    short = lambda n: n.split("(")[0].replace("void ", "").replace("cmamd::", "")
    for (s0, e0, n0), (s1, e1, n1) in zip(rows, rows[1:]):
        if prefix in n0 and prefix in n1:
            gaps.setdefault(f"{short(n0)} -> {short(n1)}", []).append((s1 - e0) / 1000.0)
    for s, e, n in rows:
        if prefix in n:
            durs.setdefault(short(n), []).append((e - s) / 1000.0)
    q = lambda a: " ".join(f"{np.percentile(a, p):7.2f}" for p in (0, 10, 50, 90, 100))
    print("gap (us, end -> next start), quantiles 0/10/50/90/100")
    for k, v in gaps.items():
        print(f"  {k:60s} n={len(v):5d}  {q(v)}")
    print("duration (us)")
    for k, v in durs.items():
        print(f"  {k:60s} n={len(v):5d}  {q(v)}")
