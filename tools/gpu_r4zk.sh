#!/bin/bash
# Round 4: mode 3 falling back to mode 1 / the bin co-run: the sampler tests, config4 under CMAMD_PIPE=3
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_sampler.py -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/r4zk_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r4zk_tests.log; [ $rc -eq 0 ] || exit $rc
CMAMD_PIPE=3 timeout -k 10 200 python bench.py --steps 100 --no-cpu-baseline --converge-seconds 0 \
  --config4-seconds 0 --config5-seconds -1 --drag-seconds -1 > gpurun_out/r4zk.json 2> gpurun_out/r4zk.err || exit $?
python -c 'import json; d=json.load(open("gpurun_out/r4zk.json")); c=d["config4_fast21"]; print("mode 3: headline", round(d["value"]/1e6,3), "config4", round(c["ms_per_step"]*1e3,2), c["kernel_us_per_step"])'
