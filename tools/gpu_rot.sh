#!/bin/bash
# rotation parity (parallel vs serial path, reference chains, C oracle), sampler + checkpoint tests, config4 trace, stamps
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_sampler.py tests/test_gpu_checkpoint.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/gpu_rot_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/gpu_rot_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_c4trace.sh && cat gpurun_out/c4_summary.txt || exit 1
timeout -k 10 300 python3 tools/mh_stamps_c4.py > gpurun_out/c4_stamps.txt 2>&1; rc=$?; head -6 gpurun_out/c4_stamps.txt; exit $rc
