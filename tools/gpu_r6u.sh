#!/bin/bash
# The drag stages writing back only the RANMAR entries their draws overwrote:
# the sampler GPU tests, then A/B of the drag leg against the previous build
# (tools/_alt_base).
set -u
mkdir -p gpurun_out/r6u
export PYTHONUNBUFFERED=1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_sampler.py tests/test_gpu_checkpoint.py -m gpu -x -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r6u/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r6u/tests.log; [ $rc -eq 0 ] || exit $rc
REPS=3 BENCH_ARGS="--steps 20 --warmup 5 --no-cpu-baseline --cache-steps -1 --converge-seconds 0 --config1-seconds -1 --config4-seconds -1 --config5-seconds -1 --drag-seconds 3" \
  tools/gpu_ab_env.sh "base" "COSMOMC_AMD_LIB=tools/_alt_base/libcosmomc_amd.so"
