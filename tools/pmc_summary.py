#!/usr/bin/env python3
"""Average per-launch PMC values per library kernel from rocprofv3 --pmc passes.

Derived figures (MI355X_MICROARCH.md, HBM and PMC-unit sections):
  hbm bytes   = 2 * 1024 * FETCH_SIZE (KB, halved on gfx950) + 1024 * WRITE_SIZE
  clock cyc   = GRBM_GUI_ACTIVE / 8   (summed over the 8 XCDs)
  mfma util   = SQ_VALU_MFMA_BUSY_CYCLES / (avg duration * 2.4 GHz * 1024 SIMDs), the
                duration from the --kernel-trace --stats pass (<root>/stats/*kernel_stats.csv);
                SQ_VALU_MFMA_BUSY_CYCLES counts MFMA-pipe cycles summed over SIMDs (64 per
                f64 16x16x4, profiles/r02_mfma_f64_rate.txt); GRBM_GUI_ACTIVE / 8 reads high
                on dispatches this short, so it is reported but not used
"""
import collections
import csv
import glob
import json
import os
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(os.path.join(root, "*", "*counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("cmamd::", "").replace("void ", "")
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
dur = {}
for f in sorted(glob.glob(os.path.join(root, "*", "*kernel_stats.csv"))):
    for r in csv.DictReader(open(f)):
        k = r["Name"].split("(")[0].replace("cmamd::", "").replace("void ", "")
        dur[k] = float(r["AverageNs"]) * 1e-3
out = {}
for k, v in agg.items():
    if not any(t in k for t in ("plik", "mh_kernel", "mh_step", "mh_bin", "rot_kernel", "cmbl", "quadform", "theory")):
        continue
    avg = {c: sum(x) / len(x) for c, x in v.items()}
    rec = {"counters": {c: round(a, 1) for c, a in avg.items()}, "launches": max(len(x) for x in v.values())}
    print(k)
    for c, a in sorted(avg.items()):
        print(f"    {c:28s} {a:14.0f}")
    if "FETCH_SIZE" in avg:
        rec["fetch_bytes"] = 2 * 1024 * avg["FETCH_SIZE"]
    if "WRITE_SIZE" in avg:
        rec["write_bytes"] = 1024 * avg["WRITE_SIZE"]
    if k in dur:
        rec["kernel_us"] = dur[k]
        print(f"    {'avg duration (us)':28s} {dur[k]:14.2f}")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in avg:
            rec["mfma_f64_16x16x4"] = avg["SQ_VALU_MFMA_BUSY_CYCLES"] / 64
            rec["mfma_busy_frac"] = avg["SQ_VALU_MFMA_BUSY_CYCLES"] / (dur[k] * 1e-6 * 2.4e9 * 1024)
            rec["mfma_tflops"] = rec["mfma_f64_16x16x4"] * 2048 / (dur[k] * 1e-6) / 1e12
            print(f"    {'f64 MFMAs (busy/64)':28s} {rec['mfma_f64_16x16x4']:14.0f}")
            print(f"    {'MFMA busy frac @2.4GHz':28s} {rec['mfma_busy_frac']:14.3f}")
            print(f"    {'MFMA TFLOP/s (f64)':28s} {rec['mfma_tflops']:14.2f}")
        if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
            rec["hbm_gbps"] = (rec["fetch_bytes"] + rec["write_bytes"]) / (dur[k] * 1e-6) / 1e9
            print(f"    {'HBM bytes (MB)':28s} {(rec['fetch_bytes'] + rec['write_bytes']) / 1e6:14.2f}")
            print(f"    {'HBM GB/s':28s} {rec['hbm_gbps']:14.0f}")
    out[k] = rec
if len(sys.argv) > 2:
    with open(sys.argv[2], "w") as f:
        json.dump({"walkers": int(os.environ.get("PMC_WALKERS", "1024")),
                   "note": "per-launch averages over the bench's timed and warmup steps; "
                           "fetch_bytes already doubled per the gfx950 FETCH_SIZE correction",
                   "per_launch": out}, f, indent=1)
