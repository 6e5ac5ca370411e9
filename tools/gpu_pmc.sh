#!/bin/bash
# PMC counter passes over a short bench run (one rocprofv3 run per pass, no
# tracing domains combined with --pmc).  Extra args go to bench.py.
set -u
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
timeout -k 10 120 rocprofv3 -L > "$R/gpurun_out/pmc/counters.txt" 2>&1 || true
pass() {
  name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d "$R/gpurun_out/pmc/$name" -o run \
    -- python3 "$R/bench.py" --no-cpu-baseline --steps 60 --warmup 5 $BENCH_ARGS > "$R/gpurun_out/pmc/$name.log" 2>&1
  rc=$?; echo "pmc pass $name rc=$rc"; return $rc
}
BENCH_ARGS="${BENCH_ARGS:-}"
pass sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE && \
pass fetch FETCH_SIZE && \
pass write WRITE_SIZE TCC_HIT_sum && \
pass l2 TCC_HIT_sum TCC_MISS_sum SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE && \
pass inst SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_INSTS_MFMA && \
pass inst2 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR
