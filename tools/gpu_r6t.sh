#!/bin/bash
# rocprofv3 kernel statistics of the dragging leg (config2_drag) alone.
set -u
mkdir -p gpurun_out/r6t
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/r6t/prof" -o run \
  -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --cache-steps -1 --converge-seconds 0 \
  --config1-seconds -1 --config4-seconds -1 --config5-seconds -1 --drag-seconds 0 > "$R/gpurun_out/r6t/prof.log" 2>&1
rc=$?; echo "prof rc=$rc"; rm -f "$R"/gpurun_out/r6t/prof/*kernel_trace.csv; exit $rc
