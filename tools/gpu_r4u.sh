#!/bin/bash
# Round 4: bin co-run with Delta from the raw sums + ksplit; config4 leg
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_sampler.py -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "bin_corun or plik_fast or rotation or giveup or pipelined" > gpurun_out/r4u_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r4u_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 50 --no-cpu-baseline --converge-seconds 0 --config4-seconds 0 \
  --config5-seconds -1 --drag-seconds -1 > gpurun_out/r4u.json 2> gpurun_out/r4u.err
rc=$?; [ $rc -eq 0 ] || { tail -20 gpurun_out/r4u.err; exit $rc; }
python -c 'import json; d=json.load(open("gpurun_out/r4u.json")); c=d["config4_fast21"]; print("config4", round(c["ms_per_step"]*1e3,2), "us/step", c["avg_kernel_us"], c["kernel_us_per_step"])'
