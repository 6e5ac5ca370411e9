#!/bin/bash
# A/B of the quadratic form's column-block chunk (CMAMD_QF_KB) on the
# configs[1], configs[3] and configs[4] legs.
set -u
export PYTHONUNBUFFERED=1
REPS=2 BENCH_ARGS="--steps 20 --warmup 5 --no-cpu-baseline --cache-steps -1 --converge-seconds 0 --config1-seconds 3 --config4-seconds 4 --config5-seconds 4 --drag-seconds -1" \
  tools/gpu_ab_env.sh "base" "CMAMD_QF_KB=1" "CMAMD_QF_KB=3" "CMAMD_QF_KB=4"
