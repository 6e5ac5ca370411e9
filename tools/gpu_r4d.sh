#!/bin/bash
# Round 4: Metropolis phase cycles alone (mode 0: mh_kernel, mode 2: mh_kernel
# between step tails) and beside the pass (mode 1: mh_pass_kernel, mode 4:
# mh_half_kernel).
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for m in 0 2 1 4; do
  echo "== mode $m"
  CMAMD_PIPE=$m timeout -k 10 120 python tools/mh_stamps.py --no-build > gpurun_out/r4d_mh_m$m.txt 2>&1
  rc=$?; grep -v amdgpu.ids gpurun_out/r4d_mh_m$m.txt; [ $rc -eq 0 ] || exit $rc
done
