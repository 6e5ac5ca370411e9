#!/bin/bash
# Round 6: PMC passes over the configs[1] (plik_lite TT, W = 256) and
# configs[4] (BK15 + plik_lite) legs alone, for the per-kernel attribution.
set -u
PMC_OUT=${PMC_OUT:-r6b_legs} PMC_BENCH_ARGS="--no-cpu-baseline --steps 2 --warmup 1 --cache-steps -1 --converge-seconds 0 \
--config1-seconds 0 --config4-seconds -1 --config5-seconds 0 --drag-seconds -1" tools/gpu_pmc.sh
