#!/bin/bash
# A/B: the unified launch's pass role with the two-step weight prefetch
# (-DCMAMD_UNI_W2=1, tools/_altuw2) at 352-l items.
set -u
export PYTHONUNBUFFERED=1
REPS=3 tools/gpu_ab_env.sh "base" "COSMOMC_AMD_LIB=tools/_altuw2/libcosmomc_amd.so"
