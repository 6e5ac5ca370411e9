#!/bin/bash
set -u
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out/c4"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/c4" -o run \
  -- python3 "$R/tools/c4_trace.py" > "$R/gpurun_out/c4/run.log" 2>&1 || exit $?
python3 "$R/tools/c4_trace.py" --summary "$R/gpurun_out/c4/run_kernel_trace.csv" > "$R/gpurun_out/c4_summary.txt" || exit 1
if [ -n "${C4_BOTH:-}" ]; then
  mkdir -p "$R/gpurun_out/c4b"
  C4_STAGE_R=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/c4b" -o run \
    -- python3 "$R/tools/c4_trace.py" > "$R/gpurun_out/c4b/run.log" 2>&1 || exit $?
  python3 "$R/tools/c4_trace.py" --summary "$R/gpurun_out/c4b/run_kernel_trace.csv" > "$R/gpurun_out/c4b_summary.txt"
fi
