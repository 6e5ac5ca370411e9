#!/bin/bash
# Round 4: shorter Metropolis chain (two-phase test rows, batched scaling, no re-copy after accept)
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_sampler.py -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/r4n_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4n_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/mh_stamps_c4.py > gpurun_out/r4n_c4_stamps.txt 2>&1 || exit $?
sed -n '1,3p;18,26p' gpurun_out/r4n_c4_stamps.txt
timeout -k 10 300 python bench.py --steps 100 --no-cpu-baseline --converge-seconds 0 --config4-seconds 0 \
  --config5-seconds -1 --drag-seconds -1 > gpurun_out/r4n.json 2> gpurun_out/r4n.err
rc=$?; [ $rc -eq 0 ] || { tail -20 gpurun_out/r4n.err; exit $rc; }
python -c 'import json; d=json.load(open("gpurun_out/r4n.json")); c=d["config4_fast21"]; print("config4", round(c["ms_per_step"]*1e3,2), "us/step", c["avg_kernel_us"]); print("headline", round(d["value"]/1e6,3), round(d["ms_per_step"]*1e3,2), d["roofline"]["avg_kernel_us"])'
