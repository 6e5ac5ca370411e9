#!/bin/bash
# A/B of the BK prologue's workgroup size (CMAMD_BKP_THREADS, 256 in tree: a
# wave per map at a time) on the configs[4] leg.
set -u
export PYTHONUNBUFFERED=1
V=""
for a in ${ALTS:-bkp128 bkp512 bkp768}; do V="$V COSMOMC_AMD_LIB=tools/_alt_$a/libcosmomc_amd.so"; done
REPS=2 BENCH_ARGS="--steps 20 --warmup 5 --no-cpu-baseline --cache-steps -1 --converge-seconds 0 --config1-seconds -1 --config4-seconds -1 --config5-seconds 4 --drag-seconds -1" \
  tools/gpu_ab_env.sh "base" $V
