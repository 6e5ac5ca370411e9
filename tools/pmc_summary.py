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
for k, v in agg.items():
    if any(t in k for t in ("plik", "mh_kernel")):
        print(k)
        for c, x in sorted(v.items()):
            print(f"    {c:28s} {sum(x) / len(x):14.0f}")
