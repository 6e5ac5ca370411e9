#!/usr/bin/env python3
"""Average per-launch PMC values per kernel from tools/gpu_pmc.sh output."""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(os.path.join(root, "*", "*counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("cmamd::", "").replace("void ", "")
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
traffic = {}
for k, v in agg.items():
    if any(t in k for t in ("plik", "mh_kernel", "rot_kernel", "cmbl", "quadform", "theory")):
        print(k)
        for c, x in sorted(v.items()):
            print(f"    {c:28s} {sum(x) / len(x):14.0f}")
        avg = {c: sum(x) / len(x) for c, x in v.items()}
        if "FETCH_SIZE" in avg:
            # MI355X_MICROARCH.md "HBM [CDNA4]": FETCH_SIZE (KB) reports half the bytes of
            # 16-B/lane streaming reads on gfx950 -> x2; WRITE_SIZE (KB) is exact
            traffic[k] = {"fetch_bytes": 2 * 1024 * avg["FETCH_SIZE"],
                          "write_bytes": 1024 * avg.get("WRITE_SIZE", 0.0)}
if len(sys.argv) > 2:
    import json
    with open(sys.argv[2], "w") as f:
        json.dump({"walkers": int(os.environ.get("PMC_WALKERS", "1024")), "per_launch": traffic}, f, indent=1)
