#!/bin/bash
# A/B: BK15's quadratic form with 2 column blocks per item (CMAMD_QF_KB=2
# leaves plik_lite's choice, 2, unchanged; BK15's pick is 3) on configs[4].
set -u
export PYTHONUNBUFFERED=1
REPS=3 BENCH_ARGS="--steps 20 --warmup 5 --no-cpu-baseline --cache-steps -1 --converge-seconds 0 --config1-seconds -1 --config4-seconds -1 --config5-seconds 4 --drag-seconds -1" \
  tools/gpu_ab_env.sh "base" "CMAMD_QF_KB=2"
