#!/bin/bash
# Round 4: the chain maps narrow blocks itself (no group mapping phase): sampler tests, headline, config4
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_sampler.py -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/r4za_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r4za_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 300 --no-cpu-baseline --converge-seconds 0 --config4-seconds 0 \
  --config5-seconds -1 --drag-seconds -1 > gpurun_out/r4za_$i.json 2> gpurun_out/r4za_$i.err || exit $?
python -c 'import json,sys; d=json.load(open(sys.argv[1])); c=d["config4_fast21"]; print("config4", round(c["ms_per_step"]*1e3,2), c["kernel_us_per_step"]); print("headline", round(d["value"]/1e6,3), round(d["ms_per_step"]*1e3,2), d["roofline"]["avg_kernel_us"])' gpurun_out/r4za_$i.json
done
