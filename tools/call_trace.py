#!/usr/bin/env python3
"""Per-launch timeline of the headline's fast-step calls from a rocprofv3
kernel trace of the driver's bench command:
    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ct -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 ...
    python3 tools/call_trace.py gpurun_out/ct/run_kernel_trace.csv
A call is a run of mh_* launches with no gap above 40 us; for each call it
prints the launch count, span, summed kernel time, summed inter-launch gaps
and the per-launch durations in order (which show a clock or cache ramp)."""
import csv
import sys


def main(path):
    rows = []
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("cmamd::", "")
        if k.startswith("mh_"):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), k))
    rows.sort()
    calls, cur = [], []
    for s, e, k in rows:
        if cur and s - cur[-1][1] > 40_000:
            calls.append(cur)
            cur = []
        cur.append((s, e, k))
    if cur:
        calls.append(cur)
    for i, c in enumerate(calls):
        durs = [(e - s) * 1e-3 for s, e, _ in c]
        gaps = [(c[j + 1][0] - c[j][1]) * 1e-3 for j in range(len(c) - 1)]
        span = (c[-1][1] - c[0][0]) * 1e-3
        print(f"call {i}: {len(c)} launches, span {span:.1f} us, kernels {sum(durs):.1f} us, gaps {sum(gaps):.1f} us "
              f"(max {max(gaps) if gaps else 0:.1f})")
        print("   durations:", " ".join(f"{d:.1f}" for d in durs))
        if gaps:
            print("   gaps:     ", " ".join(f"{g:.1f}" for g in gaps))


if __name__ == "__main__":
    main(sys.argv[1])
