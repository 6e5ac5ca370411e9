#!/bin/bash
# Round-3 counter evidence for the headline workload: one kernel-trace --stats
# run, then three --pmc passes of their own (MFMA busy + clocks, FETCH_SIZE,
# WRITE_SIZE), summarised by tools/pmc_summary.py; per-dispatch CSVs deleted.
set -u
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out/pmc"
cd /tmp && export TMPDIR=/tmp
ARGS="--no-cpu-baseline --steps 60 --warmup 5 --converge-seconds 0 --config4-seconds -1 --config5-seconds -1 --drag-seconds -1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/pmc/stats" -o run \
  -- python3 "$R/bench.py" $ARGS > "$R/gpurun_out/pmc/stats.log" 2>&1 || exit $?
for pass in "sq SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE" "fetch FETCH_SIZE" "write WRITE_SIZE"; do
  set -- $pass
  name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d "$R/gpurun_out/pmc/$name" -o run \
    -- python3 "$R/bench.py" $ARGS > "$R/gpurun_out/pmc/$name.log" 2>&1 || exit $?
done
cd "$R" && PMC_WALKERS=1024 python3 tools/pmc_summary.py gpurun_out/pmc gpurun_out/pmc_traffic.json > gpurun_out/pmc_summary.txt
rc=$?
cp gpurun_out/pmc/stats/*kernel_stats.csv gpurun_out/kernel_stats.csv 2>/dev/null
rm -rf gpurun_out/pmc/sq gpurun_out/pmc/fetch gpurun_out/pmc/write gpurun_out/pmc/stats/*kernel_trace.csv
exit $rc
