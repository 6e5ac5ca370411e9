#!/bin/bash
set -u
mkdir -p gpurun_out/fold
export PYTHONUNBUFFERED=1
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_sampler.py -k "pipelined_steps_bitwise or handoff_giveup" > gpurun_out/fold/tests.log 2>&1; rc=$?; tail -2 gpurun_out/fold/tests.log; [ $rc -eq 0 ] || exit $rc
REPS=2 bash tools/gpu_ab_env.sh "CMAMD_PIPE=3 CMAMD_FOLD_G=1" "CMAMD_PIPE=3 CMAMD_FOLD_G=0" "CMAMD_PIPE=1"
