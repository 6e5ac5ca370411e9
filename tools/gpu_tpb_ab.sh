#!/bin/bash
# fused-pass item plan: balanced per-field cuts (CMAMD_TP_BALANCE=1) against the greedy TP_MAXL grouping
set -u
mkdir -p gpurun_out
ARGS="--no-cpu-baseline --steps 400 --warmup 20 --converge-seconds 0 --config4-seconds -1 --config5-seconds -1 --drag-seconds -1"
for rep in 1 2; do for v in 1 0; do
  CMAMD_TP_BALANCE=$v timeout -k 10 300 python bench.py $ARGS > gpurun_out/tpb_$v.json 2> gpurun_out/tpb_$v.err || { tail -5 gpurun_out/tpb_$v.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/tpb_$v.json').read().strip().splitlines()[-1])
print('balance=$v', round(d['value']/1e6,3), 'M', round(d['ms_per_step']*1e3,2), 'us/step', round(d['roofline']['avg_kernel_us']['theory_window_kernel'],2))"
done; done
