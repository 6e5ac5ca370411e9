#!/bin/bash
# HBM traffic per launch of every library kernel at the bench's headline
# workload (FETCH_SIZE x2 + WRITE_SIZE per the MI355X guide), two rocprofv3
# --pmc passes of their own, summarised into gpurun_out/pmc_traffic.json;
# the per-dispatch CSVs are deleted (they exceed the copy-back limit).
set -u
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out/pmc"
cd /tmp && export TMPDIR=/tmp
for pass in "fetch FETCH_SIZE" "write WRITE_SIZE"; do
  set -- $pass
  timeout -k 10 300 rocprofv3 --pmc $2 --output-format csv -d "$R/gpurun_out/pmc/$1" -o run \
    -- python3 "$R/bench.py" --no-cpu-baseline --steps 60 --warmup 5 --converge-seconds 0 --config4-seconds -1 \
       --config5-seconds -1 --drag-seconds -1 > "$R/gpurun_out/pmc/$1.log" 2>&1 || exit $?
done
cd "$R" && PMC_WALKERS=1024 python3 tools/pmc_summary.py gpurun_out/pmc gpurun_out/pmc_traffic.json > gpurun_out/pmc_summary.txt
rc=$?
rm -rf gpurun_out/pmc/fetch gpurun_out/pmc/write
exit $rc
