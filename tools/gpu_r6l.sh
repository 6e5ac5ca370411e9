#!/bin/bash
# A/B: the quadratic form's column-block chunk per item (CMAMD_QF_KB; the
# chosen default is 2 for plik_lite) and the tail wait's poll sleep
# (-DCMAMD_TW_SLEEP, 20 in tree) in the unified launch.
set -u
export PYTHONUNBUFFERED=1
REPS=${REPS:-2} tools/gpu_ab_env.sh "base" "CMAMD_QF_KB=1" "CMAMD_QF_KB=3" \
  "COSMOMC_AMD_LIB=tools/_alttw8/libcosmomc_amd.so" "COSMOMC_AMD_LIB=tools/_alttw40/libcosmomc_amd.so"
