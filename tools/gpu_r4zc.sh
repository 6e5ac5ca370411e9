#!/bin/bash
# Round 4: every kernel of the drag leg (rocprofv3 --kernel-trace --stats)
set -u
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out/dragprof"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/dragprof" -o run \
  -- python3 "$R/bench.py" --steps 20 --warmup 2 --no-cpu-baseline --converge-seconds 0 --config4-seconds -1 \
     --config5-seconds -1 --drag-seconds 0 > "$R/gpurun_out/dragprof/run.log" 2>&1
rc=$?; rm -f "$R"/gpurun_out/dragprof/*kernel_trace.csv; exit $rc
