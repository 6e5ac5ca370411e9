#!/bin/bash
# Round 4: rotation rows in HBM for config4_fast21 (tests, mh phase cycles staged vs in place, the leg)
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_sampler.py -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/r4j_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4j_tests.log; [ $rc -eq 0 ] || exit $rc
for m in 1 0; do
  C4_STAGE_R=$m timeout -k 10 200 python -u tools/mh_stamps_c4.py > gpurun_out/r4j_c4_stamps_R$m.txt 2>&1 || exit $?
  echo "stage_R=$m"; sed -n '1,3p;20,24p' gpurun_out/r4j_c4_stamps_R$m.txt
done
timeout -k 10 300 python bench.py --steps 50 --no-cpu-baseline --converge-seconds 0 --config4-seconds 0 \
  --config5-seconds -1 --drag-seconds -1 > gpurun_out/r4j.json 2> gpurun_out/r4j.err
rc=$?; [ $rc -eq 0 ] || { tail -20 gpurun_out/r4j.err; exit $rc; }
python -c 'import json; d=json.load(open("gpurun_out/r4j.json")); c=d["config4_fast21"]; print("config4", round(c["ms_per_step"]*1e3,2), "us/step", c["avg_kernel_us"]); print("headline", round(d["value"]/1e6,3))'
