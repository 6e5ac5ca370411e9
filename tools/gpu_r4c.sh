#!/bin/bash
# Round 4: interleaved halves (mode 4) and the unified launch with a persistent
# pass under several role orders: schedule tests, bench, block timelines.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests/test_gpu_sampler.py -x -v --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "pipelined" > gpurun_out/r4c_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4c_tests.log; [ $rc -eq 0 ] || exit $rc
COSMOMC_AMD_LIB=$PWD/tools/_mb8/libcosmomc_amd.so timeout -k 10 600 python -u -m pytest tests/test_gpu_sampler.py -x -v \
  --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4c_tests_mb8.log 2>&1
rc=$?; tail -3 gpurun_out/r4c_tests_mb8.log; [ $rc -eq 0 ] || exit $rc
run() {   # mode order persist tag [lib]
  COSMOMC_AMD_LIB=${5:-} CMAMD_PIPE=$1 CMAMD_TAIL_ORDER=$2 CMAMD_PASS_PERSIST=$3 timeout -k 10 200 python bench.py --steps 300 --no-cpu-baseline \
    --converge-seconds 0 --config4-seconds -1 --config5-seconds -1 --drag-seconds -1 > gpurun_out/r4c_$4.json 2> gpurun_out/r4c_$4.err
  rc=$?; [ $rc -eq 0 ] || { echo "$4 rc=$rc"; tail -5 gpurun_out/r4c_$4.err; return $rc; }
  python - "$4" <<'PY'
import json, sys
d = json.load(open(f"gpurun_out/r4c_{sys.argv[1]}.json"))
print(sys.argv[1], round(d["value"] / 1e6, 3), "M evals/s", round(d["ms_per_step"] * 1e3, 2), "us/step",
      {k: round(v, 2) for k, v in d["roofline"]["avg_kernel_us"].items() if v})
PY
}
MB8=$PWD/tools/_mb8/libcosmomc_amd.so
run 4 qgp 0 m4_qgp && run 4 pqg 0 m4_pqg && run 4 qgp 0 m4_qgp_mb8 $MB8 && run 3 pqg 1 m3_pqg_P && run 3 gqp 1 m3_gqp_P && \
run 3 'p*qg' 1 m3_pxq_P && run 3 gqp 0 m3_gqp && run 1 qpg 0 m1 && run 1 qpg 0 m1_mb8 $MB8 && run 3 gqp 0 m3_gqp_mb8 $MB8 || exit 1
for o in pqg gqp; do
  CMAMD_PASS_PERSIST=1 CMAMD_TAIL_ORDER=$o timeout -k 10 150 python tools/uni_stamps.py --no-build > gpurun_out/r4c_stamps_$o.txt 2>&1
  rc=$?; grep -v amdgpu.ids gpurun_out/r4c_stamps_$o.txt; [ $rc -eq 0 ] || exit $rc
done
