#!/bin/bash
# Round 4: ROT_DEFER_MIN 4 (config5's 7-wide block in rot_kernel): sampler tests, config4/config5 legs
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_sampler.py -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/r4y_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r4y_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 50 --no-cpu-baseline --converge-seconds 0 --config4-seconds 0 \
  --config5-seconds -1 --drag-seconds -1 > gpurun_out/r4y.json 2> gpurun_out/r4y.err
rc=$?; [ $rc -eq 0 ] || { tail -20 gpurun_out/r4y.err; exit $rc; }
python -c 'import json; d=json.load(open("gpurun_out/r4y.json")); c=d["config4_fast21"]; print("config4", round(c["ms_per_step"]*1e3,2), c["kernel_us_per_step"]); print("headline", round(d["value"]/1e6,3))'
