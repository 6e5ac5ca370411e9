#!/bin/bash
# Per-call fixed cost of the step call (tools/call_overhead.py) and the gaps
# between the unified launches from a rocprofv3 kernel trace (tools/kernel_gaps.py).
set -u
mkdir -p gpurun_out/r6h
export PYTHONUNBUFFERED=1
timeout -k 10 300 python3 tools/call_overhead.py > gpurun_out/r6h/overhead.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/r6h/overhead.txt; [ $rc -eq 0 ] || exit $rc
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/r6h/trace" -o run \
  -- python3 "$R/bench.py" --steps 100 --warmup 5 --no-cpu-baseline --cache-steps -1 --converge-seconds 0 \
  --config1-seconds -1 --config4-seconds -1 --config5-seconds -1 --drag-seconds -1 > "$R/gpurun_out/r6h/trace.log" 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd "$R"
python3 tools/kernel_gaps.py gpurun_out/r6h/trace/run_kernel_trace.csv | tee gpurun_out/r6h/gaps.txt
