#!/bin/bash
# A/B of the window pass with its weight tiles fetched two steps ahead
# (-DCMAMD_TP_W2=1, tools/_alt) against the in-tree build: the sampler and
# plik GPU tests on the variant, then interleaved headline + drag benches.
set -u
mkdir -p gpurun_out/r6i
export PYTHONUNBUFFERED=1
ALT=tools/_alt/libcosmomc_amd.so
COSMOMC_AMD_LIB=$ALT timeout -k 10 600 python3 -u -m pytest tests/test_gpu_sampler.py tests/test_gpu_plik.py -m gpu -x -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r6i/tests_alt.log 2>&1
rc=$?; echo "alt pytest rc=$rc"; tail -2 gpurun_out/r6i/tests_alt.log; [ $rc -eq 0 ] || exit $rc
REPS=3 BENCH_ARGS="--steps 300 --warmup 20 --no-cpu-baseline --cache-steps -1 --converge-seconds 0 --config1-seconds -1 --config4-seconds -1 --config5-seconds -1 --drag-seconds 3" \
  tools/gpu_ab_env.sh "base" "COSMOMC_AMD_LIB=$ALT"
