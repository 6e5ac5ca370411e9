#!/bin/bash
# A/B of the theory pass variants (CMAMD_TP_VEC): fused-pass tests, then a quick headline bench per variant
set -u
mkdir -p gpurun_out
ARGS="--no-cpu-baseline --steps 300 --warmup 20 --converge-seconds 0 --config4-seconds -1 --config5-seconds -1 --drag-seconds -1"
for v in ${TP_VARIANTS:-1 0}; do
  CMAMD_TP_VEC=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_sampler.py tests/test_gpu_cmblikes.py -x -q --timeout 120 --timeout-method thread \
     -p no:cacheprovider -k "fused_window_pass or deferred_combine or fused or drag" > gpurun_out/tp_ab_test_$v.log 2>&1 || { echo "tests v=$v failed"; tail -30 gpurun_out/tp_ab_test_$v.log; exit 1; }
  tail -1 gpurun_out/tp_ab_test_$v.log
  CMAMD_TP_VEC=$v timeout -k 10 300 python bench.py $ARGS > gpurun_out/tp_ab_$v.json 2> gpurun_out/tp_ab_$v.err || { echo "bench v=$v failed"; tail -5 gpurun_out/tp_ab_$v.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/tp_ab_$v.json').read().strip().splitlines()[-1])
print('v=$v', round(d['value']/1e6,3), 'M', round(d['ms_per_step']*1e3,2), 'us/step', d['roofline']['avg_kernel_us'])"
done
