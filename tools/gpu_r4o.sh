#!/bin/bash
# Round 4: config4_fast21 leg, per-kernel split
set -u
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 50 --no-cpu-baseline --converge-seconds 0 --config4-seconds 0 \
  --config5-seconds -1 --drag-seconds -1 > gpurun_out/r4o.json 2> gpurun_out/r4o.err
rc=$?; [ $rc -eq 0 ] || { tail -20 gpurun_out/r4o.err; exit $rc; }
python -c 'import json; d=json.load(open("gpurun_out/r4o.json")); c=d["config4_fast21"]; print("config4", round(c["ms_per_step"]*1e3,2), "us/step", c["avg_kernel_us"], c["kernel_us_per_step"])'
