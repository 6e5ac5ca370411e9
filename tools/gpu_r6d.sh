#!/bin/bash
# Round 6: configs[4] (BK15 + plik_lite) -- the window group kernel's
# tile-per-XCD placement and the prologue's spread integrals -- checked by the
# CMBlikes / BK / sampler GPU tests, then timed (interleaved A/B of the
# placement) with the headline's two-step-ahead quadratic form as default.
set -u
mkdir -p gpurun_out/r6d
export PYTHONUNBUFFERED=1
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_cmblikes.py tests/test_gpu_sampler.py tests/test_gpu_smica.py -m gpu -x -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r6d/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r6d/tests.log; [ $rc -eq 0 ] || exit $rc
BENCH_ARGS="--steps 300 --warmup 20 --no-cpu-baseline --cache-steps -1 --converge-seconds 0 --config1-seconds -1 --config4-seconds -1 --config5-seconds 0 --drag-seconds -1" \
  REPS=2 tools/gpu_ab_env.sh "base" "CMAMD_WG_MAP=0" "CMAMD_QF_AHEAD=0" || exit $?
