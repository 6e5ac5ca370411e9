#!/bin/bash
# A/B of the window pass's item length (CMAMD_TP_MAXL, l per work item; 288 in
# tree) inside the unified launch and the standalone drag pass.
set -u
mkdir -p gpurun_out/r6j
export PYTHONUNBUFFERED=1
V=""
for L in ${ALTS:-352 384 416 448 480}; do V="$V COSMOMC_AMD_LIB=tools/_alt$L/libcosmomc_amd.so"; done
REPS=${REPS:-2} BENCH_ARGS="--steps 300 --warmup 20 --no-cpu-baseline --cache-steps -1 --converge-seconds 0 --config1-seconds -1 --config4-seconds -1 --config5-seconds -1 --drag-seconds 3" \
  tools/gpu_ab_env.sh "base" $V
