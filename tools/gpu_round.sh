#!/bin/bash
# GPU-box session: the whole -m gpu suite, then a short headline bench (no
# side legs), then the mh_kernel stamps.  Every GPU step has its own limit;
# the first failure ends it.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --converge-seconds 0 --config4-seconds -1 --config5-seconds -1 --drag-seconds -1 > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err
rc=$?; echo "bench rc=$rc"; python -c "
import json; d=json.load(open('gpurun_out/bench_quick.json')); print(d['value'], d['ms_per_step'], d['roofline']['avg_kernel_us'])"
[ $rc -eq 0 ] || exit $rc
if [ "${STAMPS:-1}" = "1" ]; then
  timeout -k 10 120 python tools/mh_stamps.py --no-build > gpurun_out/mh_stamps.txt 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/mh_stamps.txt
fi
exit $rc
