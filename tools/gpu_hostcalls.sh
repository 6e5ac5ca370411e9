#!/bin/bash
# Host-side cost of one 20-step headline call: HIP API trace + kernel trace of
# the driver's bench command, then the API calls between the timed call's
# launches (tools/host_trace.py)
set -u
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/hostcalls"
mkdir -p "$OUT"
NB="--no-cpu-baseline --converge-seconds 0 --config1-seconds -1 --config4-seconds -1 --config5-seconds -1 --drag-seconds -1"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d "$OUT/tr" -o run \
  -- python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5 $NB > "$OUT/trace_bench.json" 2>/dev/null || exit $?
ls "$OUT/tr" > "$OUT/files.txt"
python3 "$R/tools/host_trace.py" "$OUT/tr" | tee "$OUT/host.txt"
rm -f "$OUT"/tr/*.csv
