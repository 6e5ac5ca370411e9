#!/bin/bash
# config5 (BK15 + plik) HL kernel time with and without the warm-started eigensolves
set -u
mkdir -p gpurun_out
for v in 3 0; do
  CMAMD_HL_WARM=$v timeout -k 10 300 python bench.py --steps 50 --no-cpu-baseline --converge-seconds 0 --config4-seconds -1 --config5-seconds 0 --drag-seconds -1 > gpurun_out/bench_hl_$v.json 2> gpurun_out/bench_hl_$v.err || exit 1
  python -c "
import json; d=json.load(open('gpurun_out/bench_hl_$v.json')); c=d['config5_bk15_plik']; print('warm=$v', round(c['evals_per_s']/1e6,3), round(c['ms_per_step']*1e3,1), c['avg_kernel_us']['cmbl_hl_kernel'])"
done
