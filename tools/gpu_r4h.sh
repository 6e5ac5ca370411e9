#!/bin/bash
# Round 4: configs[3] / configs[4] legs' step times and per-kernel averages.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python bench.py --steps 50 --no-cpu-baseline --converge-seconds 0 --config4-seconds 0 \
  --config5-seconds 0 --drag-seconds -1 > gpurun_out/r4h.json 2> gpurun_out/r4h.err
rc=$?; [ $rc -eq 0 ] || { tail -20 gpurun_out/r4h.err; exit $rc; }
python - <<'PY'
import json; d=json.load(open("gpurun_out/r4h.json"))
for k in ("config4_fast21", "config5_bk15_plik"):
    c = d[k]; print(k, round(c["ms_per_step"]*1e3, 2), "us/step", c["avg_kernel_us"])
PY
