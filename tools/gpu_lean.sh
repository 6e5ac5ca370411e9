#!/bin/bash
# lean chain + per-problem HL stop: the schedule / determinism tests, an interleaved A/B, stamps
set -u
mkdir -p gpurun_out/lean
export PYTHONUNBUFFERED=1
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_sampler.py tests/test_gpu_cmblikes.py -k "pipelined_steps_bitwise or plik_fast_chain or pipelined_with_wide or handoff_giveup or config5_joint or walker_order or hl_every or golden" > gpurun_out/lean/tests.log 2>&1; rc=$?; tail -3 gpurun_out/lean/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/ab_steps.py --steps 300 --reps 2 > gpurun_out/lean/ab.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/lean/ab.log; [ $rc -eq 0 ] || exit $rc
STAMP_OUT=$PWD/tools/_stamped timeout -k 10 120 python3 tools/mh_stamps.py --no-build > gpurun_out/lean/stamps.txt 2>&1; grep -v amdgpu.ids gpurun_out/lean/stamps.txt
