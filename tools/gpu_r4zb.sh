#!/bin/bash
# Round 4: the quadratic form's K split (CMAMD_QF_KB) at W = 512 (config4) and W = 1024 (headline)
set -u
mkdir -p gpurun_out
for kb in 0 1 2 3 4 5; do
  CMAMD_QF_KB=$kb timeout -k 10 200 python bench.py --steps 200 --no-cpu-baseline --converge-seconds 0 --config4-seconds 0 \
    --config5-seconds -1 --drag-seconds -1 > gpurun_out/r4zb_$kb.json 2> gpurun_out/r4zb_$kb.err || exit $?
  python -c 'import json,sys; d=json.load(open(sys.argv[1])); c=d["config4_fast21"]; print("kb", sys.argv[2], "config4", round(c["ms_per_step"]*1e3,2), c["kernel_us_per_step"].get("plik_quadform_ksplit"), "headline", round(d["ms_per_step"]*1e3,2), d["roofline"]["avg_kernel_us"])' gpurun_out/r4zb_$kb.json $kb
done
