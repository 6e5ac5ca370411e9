#!/bin/bash
# Round 4: HL Jacobi with two columns a lane and DPP ring moves: tests, then the config5 leg
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_cmblikes.py tests/test_gpu_sampler.py -x -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider -k "hl or HL or bk or BK or config5 or cmbl" > gpurun_out/r4w_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4w_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 50 --no-cpu-baseline --converge-seconds 0 --config4-seconds -1 \
  --config5-seconds 0 --drag-seconds -1 > gpurun_out/r4w.json 2> gpurun_out/r4w.err
rc=$?; [ $rc -eq 0 ] || { tail -20 gpurun_out/r4w.err; exit $rc; }
python -c 'import json; d=json.load(open("gpurun_out/r4w.json")); c=d["config5_bk15_plik"]; print("config5", round(c["ms_per_step"]*1e3,2), "us/step", c["avg_kernel_us"])'
