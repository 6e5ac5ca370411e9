#!/bin/bash
# Round 4: the unified step launch (mode 3) and the split pipelined steps
# (mode 2) against mh_pass_kernel (mode 1): the schedule tests, then the
# headline bench under each mode and role order (CMAMD_TAIL_ORDER).
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests/test_gpu_sampler.py -x -v --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "pipelined or corun or fused_window or giveup or config5" > gpurun_out/r4a_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r4a_tests.log; [ $rc -eq 0 ] || exit $rc
run() {   # mode order tag
  CMAMD_PIPE=$1 CMAMD_TAIL_ORDER=$2 timeout -k 10 200 python bench.py --steps 500 --no-cpu-baseline --converge-seconds 0 \
    --config4-seconds -1 --config5-seconds -1 --drag-seconds -1 > gpurun_out/r4a_bench_$3.json 2> gpurun_out/r4a_bench_$3.err
  rc=$?; [ $rc -eq 0 ] || { echo "$3 rc=$rc"; tail -5 gpurun_out/r4a_bench_$3.err; return $rc; }
  python - "$3" <<'PY'
import json, sys
d = json.load(open(f"gpurun_out/r4a_bench_{sys.argv[1]}.json"))
print(sys.argv[1], round(d["value"] / 1e6, 3), "M evals/s", round(d["ms_per_step"] * 1e3, 2), "us/step",
      {k: round(v, 2) for k, v in d["roofline"]["avg_kernel_us"].items() if v})
PY
}
run 3 qpg m3_qpg && run 2 qpg m2_qpg && run 1 qpg m1 && run 3 'q*pg' m3_qxp && run 3 qgp m3_qgp && \
run 2 'q*pg' m2_qxp && run 3 gqp m3_gqp && run 3 pqg m3_pqg
