#!/bin/bash
# Round 4: one accepted-theory copy per shared theory buffer: drag / theory-callback tests, the drag leg
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_sampler.py tests/test_gpu_checkpoint.py -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "drag or theory or refresh" > gpurun_out/r4ze_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r4ze_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 50 --no-cpu-baseline --converge-seconds 0 --config4-seconds -1 \
  --config5-seconds -1 --drag-seconds 0 > gpurun_out/r4ze_$i.json 2> gpurun_out/r4ze_$i.err || exit $?
python -c 'import json,sys; d=json.load(open(sys.argv[1])); c=d["config2_drag"]; print("drag", round(c["ms_per_drag_step"]*1e3,1), "us/drag step", c["kernel_us_per_drag_step"])' gpurun_out/r4ze_$i.json
done
