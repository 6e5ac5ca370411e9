#!/bin/bash
# timing ablations of theory_window_vec (CMAMD_TP_ABL: 1 no emit, 2 no MFMA, 3 neither); results invalid, timing only
set -u
mkdir -p gpurun_out
ARGS="--no-cpu-baseline --steps 300 --warmup 20 --converge-seconds 0 --config4-seconds -1 --config5-seconds -1 --drag-seconds -1"
for v in ${ABL_VARIANTS:-0 1 2 3}; do
  CMAMD_TP_ABL=$v timeout -k 10 300 python bench.py $ARGS > gpurun_out/tp_abl_$v.json 2> gpurun_out/tp_abl_$v.err || { echo "bench v=$v failed"; tail -5 gpurun_out/tp_abl_$v.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/tp_abl_$v.json').read().strip().splitlines()[-1])
print('abl=$v', d['roofline']['avg_kernel_us'])"
done
