#!/bin/bash
# bench.py over a walker-count sweep (no CPU baseline, no profiler)
set -u
mkdir -p gpurun_out
# usage: gpu_sweep.sh W... ; STREAM_GROUPS="1 2 4" sweeps stream groups too
for G in ${STREAM_GROUPS:-1}; do
for W in "$@"; do
  f=gpurun_out/sweep_W${W}_G$G
  timeout -k 10 180 python bench.py --no-cpu-baseline --walkers $W --groups $G > $f.json 2> $f.err
  rc=$?; echo "W=$W G=$G rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python -c "import json;d=json.load(open('$f.json'));print('W=$W G=$G', '%.3e evals/s'%d['value'], '%.1f us/step'%(d['ms_per_step']*1e3), {k:round(v,1) for k,v in d['roofline']['avg_kernel_us'].items() if v})"
done
done
