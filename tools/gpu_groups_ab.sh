#!/bin/bash
# headline step time with the walkers split into G stream groups (cmbs_set_groups)
set -u
mkdir -p gpurun_out
ARGS="--no-cpu-baseline --steps 300 --warmup 20 --converge-seconds 0 --config4-seconds -1 --config5-seconds -1 --drag-seconds -1"
for g in 1 2 4; do
  timeout -k 10 300 python bench.py $ARGS --groups $g > gpurun_out/grp_$g.json 2> gpurun_out/grp_$g.err || { tail -5 gpurun_out/grp_$g.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/grp_$g.json').read().strip().splitlines()[-1])
print('groups=$g', round(d['value']/1e6,3), 'M', round(d['ms_per_step']*1e3,2), 'us/step', d['roofline']['avg_kernel_us'])"
done
