#!/bin/bash
# bench.py over a walker-count sweep (no CPU baseline, no profiler)
set -u
mkdir -p gpurun_out
for W in "$@"; do
  timeout -k 10 180 python bench.py --no-cpu-baseline --walkers $W > gpurun_out/sweep_W$W.json 2> gpurun_out/sweep_W$W.err
  rc=$?; echo "W=$W rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python -c "import json;d=json.load(open('gpurun_out/sweep_W$W.json'));print(W:=$W, '%.3e evals/s'%d['value'], '%.1f us/step'%(d['ms_per_step']*1e3), {k:round(v,1) for k,v in d['roofline']['avg_kernel_us'].items() if v})"
done
