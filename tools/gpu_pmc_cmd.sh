#!/bin/bash
# PMC passes over an arbitrary python command: tools/gpu_pmc_cmd.sh <outdir> <script> [args...]
set -u
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/$1"; shift
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
pass() {
  name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- python3 "${CMD[@]}" > "$OUT/$name.log" 2>&1
  rc=$?; echo "pmc pass $name rc=$rc"; return $rc
}
CMD=("$R/$1" "${@:2}")
pass sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE && \
pass fetch FETCH_SIZE && \
pass write WRITE_SIZE TCC_HIT_sum && \
pass l2 TCC_HIT_sum TCC_MISS_sum SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE && \
pass inst SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_INSTS_MFMA
