#!/bin/bash
# persistent deferred quadratic form: parity (deferred vs in-launch combine, fused pass, sampler), then A/B timing
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_sampler.py tests/test_gpu_checkpoint.py -x -q --timeout 120 --timeout-method thread \
   -p no:cacheprovider > gpurun_out/qf_ab_test.log 2>&1 || { tail -30 gpurun_out/qf_ab_test.log; exit 1; }
tail -1 gpurun_out/qf_ab_test.log
ARGS="--no-cpu-baseline --steps 300 --warmup 20 --converge-seconds 0 --config4-seconds -1 --config5-seconds -1 --drag-seconds -1"
for v in 1 0; do
  CMAMD_QF_PERSIST=$v timeout -k 10 300 python bench.py $ARGS > gpurun_out/qf_ab_$v.json 2> gpurun_out/qf_ab_$v.err || { tail -5 gpurun_out/qf_ab_$v.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/qf_ab_$v.json').read().strip().splitlines()[-1])
print('persist=$v', round(d['value']/1e6,3), 'M', round(d['ms_per_step']*1e3,2), 'us/step', d['roofline']['avg_kernel_us'])"
done
