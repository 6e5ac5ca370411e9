#!/bin/bash
# Round 4: A/B of the default schedule (mode 1) against the unified launch (mode 3, order gqp), interleaved
set -u
mkdir -p gpurun_out
for rep in 1 2 3; do
  for m in 1 3; do
    CMAMD_PIPE=$m CMAMD_TAIL_ORDER=gqp timeout -k 10 200 python bench.py --steps 500 --no-cpu-baseline --converge-seconds 0 \
      --config4-seconds -1 --config5-seconds -1 --drag-seconds -1 > gpurun_out/r4zi_${m}_$rep.json 2> gpurun_out/r4zi_${m}_$rep.err || exit $?
    python -c 'import json,sys; d=json.load(open(sys.argv[1])); print("mode", sys.argv[2], "rep", sys.argv[3], round(d["value"]/1e6,3), "M", round(d["ms_per_step"]*1e3,2), "us/step", d["roofline"]["kernel"], d["roofline"]["frac"])' gpurun_out/r4zi_${m}_$rep.json $m $rep
  done
done
