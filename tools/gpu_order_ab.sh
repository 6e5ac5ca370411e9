#!/bin/bash
# mode 3 (unified launch) workgroup orders: the Metropolis rows last (gqp) or earlier ('m')
set -u
REPS=2 bash tools/gpu_ab_env.sh "CMAMD_PIPE=3 CMAMD_TAIL_ORDER=gqp" "CMAMD_PIPE=3 CMAMD_TAIL_ORDER=mgqp" "CMAMD_PIPE=3 CMAMD_TAIL_ORDER=gqmp" "CMAMD_PIPE=3 CMAMD_TAIL_ORDER=mqgp" "CMAMD_PIPE=3 CMAMD_TAIL_ORDER=gmq*p"
