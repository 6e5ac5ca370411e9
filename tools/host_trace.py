#!/usr/bin/env python3
"""The timed 20-step call of a rocprofv3 --kernel-trace --hip-runtime-trace
run of the headline bench (tools/gpu_hostcalls.sh): every HIP API call from
the one before the call's first mh_step launch to the last one, with its host
duration and its start relative to the call's first kernel start."""
import csv
import glob
import os
import sys


def main(d):
    kf = glob.glob(os.path.join(d, "*kernel_trace.csv"))[0]
    af = glob.glob(os.path.join(d, "*hip_api_trace.csv"))[0]
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][-40:])
                for r in csv.DictReader(open(kf)) if "mh_step" in r["Kernel_Name"])
    calls, cur = [], []
    for k in ks:
        if cur and k[0] - cur[-1][1] > 40_000:
            calls.append(cur)
            cur = []
        cur.append(k)
    calls.append(cur)
    timed = [c for c in calls if len(c) >= 15][0]   # the warmup call has fewer launches
    t0, t1 = timed[0][0], timed[-1][1]
    api = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"])
                 for r in csv.DictReader(open(af)))
    # the API calls from 300 us before the first kernel to the end of the last
    sel = [a for a in api if t0 - 300_000 <= a[0] <= t1 + 100_000]
    sel = sel[:40] + [(0, 0, '...')] + sel[-25:] if len(sel) > 70 else sel
    print(f"timed call: {len(timed)} launches, first kernel start = 0, last end {(t1 - t0) / 1e3:.1f} us")
    for s, e, f in sel:
        print(f"  {(s - t0) / 1e3:9.1f} us  {(e - s) / 1e3:7.1f} us  {f}")


if __name__ == "__main__":
    main(sys.argv[1])
