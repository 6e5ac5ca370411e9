#!/bin/bash
# Round 4: the drag leg with paired evaluation sets: tests, then the drag bench.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_sampler.py -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "drag or pipelined or walker0" > gpurun_out/r4g_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r4g_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 100 --no-cpu-baseline --converge-seconds 0 --config4-seconds -1 \
  --config5-seconds -1 --drag-seconds 0 > gpurun_out/r4g_drag.json 2> gpurun_out/r4g_drag.err
rc=$?; [ $rc -eq 0 ] || exit $rc
python -c 'import json; d=json.load(open("gpurun_out/r4g_drag.json")); c=d["config2_drag"]; print("headline", round(d["value"]/1e6,3), "M", round(d["ms_per_step"]*1e3,2), "us/step;", "drag", round(c["ms_per_drag_step"]*1e3,1), "us/drag step", c["kernel_us_per_drag_step"])'
