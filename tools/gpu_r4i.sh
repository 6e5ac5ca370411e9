#!/bin/bash
# Round 4: config4_fast21 mh_kernel phase cycles (instrumented build in tools/_stamps)
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/mh_stamps_c4.py > gpurun_out/r4i_c4_stamps.txt 2>&1
rc=$?; tail -50 gpurun_out/r4i_c4_stamps.txt; exit $rc
