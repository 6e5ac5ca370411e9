#!/bin/bash
# Round 4: the unified step launch (mode 3) and the split pipelined steps
# (mode 2) against mh_pass_kernel (mode 1): the schedule tests, then the
# headline bench under each mode.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests/test_gpu_sampler.py -x -v --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "pipelined or corun or fused_window or giveup or config5" > gpurun_out/r4a_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r4a_tests.log; [ $rc -eq 0 ] || exit $rc
for m in 3 2 1 3 2; do
  CMAMD_PIPE=$m timeout -k 10 200 python bench.py --steps 500 --no-cpu-baseline --converge-seconds 0 \
    --config4-seconds -1 --config5-seconds -1 --drag-seconds -1 > gpurun_out/r4a_bench_m$m.json 2> gpurun_out/r4a_bench_m$m.err
  rc=$?; echo "mode $m rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python - "$m" <<'PY'
import json, sys
d = json.load(open(f"gpurun_out/r4a_bench_m{sys.argv[1]}.json"))
print(sys.argv[1], round(d["value"] / 1e6, 3), "M evals/s", round(d["ms_per_step"] * 1e3, 2), "us/step",
      {k: round(v, 2) for k, v in d["roofline"]["avg_kernel_us"].items() if v})
PY
done
