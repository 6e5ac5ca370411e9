#!/bin/bash
# Instruction-fetch PMC passes (one rocprofv3 --pmc run each) over a short
# headline run: does the Metropolis chain wait on instruction fetch?
#   tools/gpu_icache.sh <outdir> [probe_steps.py args...]
set -u
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/$1"; shift
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
pass() {
  name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o run \
    -- python3 "$R/tools/probe_steps.py" $PROBE_ARGS > "$OUT/$name.log" 2>&1
  rc=$?; echo "pmc pass $name rc=$rc"; return $rc
}
PROBE_ARGS="$*"
pass ic SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES && \
pass wait SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH GRBM_GUI_ACTIVE && \
pass inst SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVES
