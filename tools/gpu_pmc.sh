#!/bin/bash
# PMC counter passes over a short headline bench run (one rocprofv3 run per
# pass, no tracing domain combined with --pmc), plus the kernel-trace --stats
# pass whose durations tools/pmc_summary.py divides by.  PMC_BENCH_ARGS replaces
# the bench arguments (e.g. the configs[1] leg alone).
set -u
OUTD=${PMC_OUT:-pmc}
mkdir -p gpurun_out/$OUTD
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
B=${PMC_BENCH_ARGS:-"--no-cpu-baseline --steps 60 --warmup 5 --cache-steps -1 --converge-seconds 0 --config1-seconds -1 --config4-seconds -1 --config5-seconds -1 --drag-seconds -1"}
pass() {
  name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d "$R/gpurun_out/$OUTD/$name" -o run \
    -- python3 "$R/bench.py" $B > "$R/gpurun_out/$OUTD/$name.log" 2>&1
  rc=$?; echo "pmc pass $name rc=$rc"; return $rc
}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/$OUTD/stats" -o run \
  -- python3 "$R/bench.py" $B > "$R/gpurun_out/$OUTD/stats.log" 2>&1 && rm -f "$R"/gpurun_out/$OUTD/stats/*kernel_trace.csv && \
pass fetch FETCH_SIZE && \
pass write WRITE_SIZE && \
pass mfma SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE && \
pass lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAVES SQ_BUSY_CYCLES
rc=$?; cd "$R"; python3 tools/pmc_summary.py gpurun_out/$OUTD gpurun_out/$OUTD/pmc_traffic.json; exit $rc
