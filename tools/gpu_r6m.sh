#!/bin/bash
# A/B of the BK window kernel's grouped items (cmbl_window_group: CMAMD_GSEG l
# per item, 256 in tree; CMAMD_GP pairs per item, 8) on the configs[4] leg.
set -u
export PYTHONUNBUFFERED=1
V=""
for a in ${ALTS:-GSEG224 G192 G224P9 G224P7}; do V="$V COSMOMC_AMD_LIB=tools/_alt_$a/libcosmomc_amd.so"; done
REPS=2 BENCH_ARGS="--steps 20 --warmup 5 --no-cpu-baseline --cache-steps -1 --converge-seconds 0 --config1-seconds -1 --config4-seconds -1 --config5-seconds 4 --drag-seconds -1" \
  tools/gpu_ab_env.sh "base" $V
