#!/bin/bash
# Round 6: the whole GPU suite on the folded chi^2 (middle launches, "mqp"),
# an interleaved A/B against the chi^2 rows and two variants, the block
# timelines, and the PMC passes of the configs[1] / configs[4] legs.
set -u
mkdir -p gpurun_out/r6c
export PYTHONUNBUFFERED=1
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/r6c/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r6c/tests.log; [ $rc -eq 0 ] || exit $rc
REPS=2 tools/gpu_ab_env.sh "base" "CMAMD_FOLD_G=0" "CMAMD_QF_AHEAD=1" "CMAMD_FOLD_LATE_PRIO=1" || exit $?
STAMP_OUT=$PWD/tools/_stamped timeout -k 10 120 python3 tools/uni_stamps.py --no-build > gpurun_out/r6c/uni_stamps.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r6c/uni_stamps.txt; [ $rc -eq 0 ] || exit $rc
CMAMD_FOLD_G=0 STAMP_OUT=$PWD/tools/_stamped timeout -k 10 120 python3 tools/uni_stamps.py --no-build > gpurun_out/r6c/uni_stamps_nofold.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r6c/uni_stamps_nofold.txt; [ $rc -eq 0 ] || exit $rc
PMC_OUT=r6c_legs tools/gpu_r6b.sh
