#!/bin/bash
# Attribution of the driver command's per-step time: the bench at warmup 5 and
# 200 (interleaved, REPS rounds), then one kernel trace of the driver command.
set -u
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/calls"
mkdir -p "$OUT"
NB="--no-cpu-baseline --converge-seconds 0 --config1-seconds -1 --config4-seconds -1 --config5-seconds -1 --drag-seconds -1"
for rep in $(seq 1 ${REPS:-2}); do
  for wu in 5 200; do
    timeout -k 10 300 python3 "$R/bench.py" --gpus 1 --steps 20 --warmup $wu $NB > "$OUT/b_${wu}_$rep.json" 2>/dev/null || exit $?
    python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print('warmup',sys.argv[2],round(d['ms_per_step']*1e3,2),'us/step',{k:round(v,2) for k,v in d['roofline']['avg_kernel_us'].items()})" "$OUT/b_${wu}_$rep.json" $wu
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/tr" -o run \
  -- python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5 $NB > "$OUT/trace_bench.json" 2>/dev/null || exit $?
python3 "$R/tools/call_trace.py" "$OUT/tr/run_kernel_trace.csv" | tee "$OUT/calls.txt"
rm -f "$OUT"/tr/*.csv
