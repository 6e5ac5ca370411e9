#!/bin/bash
# Round 4: HL sweep stop at cos 1e-4: the whole -m gpu suite, then the config5 leg
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4zg_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r4zg_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 50 --no-cpu-baseline --converge-seconds 0 --config4-seconds -1 \
  --config5-seconds 0 --drag-seconds -1 > gpurun_out/r4zg.json 2> gpurun_out/r4zg.err || exit $?
python -c 'import json; d=json.load(open("gpurun_out/r4zg.json")); c=d["config5_bk15_plik"]; print("config5", round(c["ms_per_step"]*1e3,2), "us/step", c["avg_kernel_us"])'
