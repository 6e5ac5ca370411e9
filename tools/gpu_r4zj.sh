#!/bin/bash
# Round 4: the unified launch's default row order (gqp): the pipelined tests, then CMAMD_PIPE=3 with no order set
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_sampler.py -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "pipelined or giveup" > gpurun_out/r4zj_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r4zj_tests.log; [ $rc -eq 0 ] || exit $rc
CMAMD_PIPE=3 timeout -k 10 200 python bench.py --steps 500 --no-cpu-baseline --converge-seconds 0 \
  --config4-seconds -1 --config5-seconds -1 --drag-seconds -1 > gpurun_out/r4zj.json 2> gpurun_out/r4zj.err || exit $?
python -c 'import json; d=json.load(open("gpurun_out/r4zj.json")); print("mode 3", round(d["value"]/1e6,3), "M", round(d["ms_per_step"]*1e3,2), "us/step")'
