#!/bin/bash
# Round 4: block timelines of the split (mode 2) and unified (mode 3) step launches.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for o in gqp qpg; do
  CMAMD_TAIL_ORDER=$o timeout -k 10 150 python tools/uni_stamps.py --no-build > gpurun_out/r4b_stamps_$o.txt 2>&1
  rc=$?; grep -v amdgpu.ids gpurun_out/r4b_stamps_$o.txt; [ $rc -eq 0 ] || exit $rc
done
