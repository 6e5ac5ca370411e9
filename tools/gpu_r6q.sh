#!/bin/bash
# A/B of the unified launch's row order at 352-l pass items (CMAMD_TAIL_ORDER).
set -u
export PYTHONUNBUFFERED=1
REPS=2 tools/gpu_ab_env.sh "base" "CMAMD_TAIL_ORDER=mq*p" "CMAMD_TAIL_ORDER=mpq" "CMAMD_TAIL_ORDER=qmp"
