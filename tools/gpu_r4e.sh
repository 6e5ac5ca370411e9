#!/bin/bash
# Round 4: the fused window pass with theory three steps ahead (DEPTH 3,
# occupancy 2) against the default (two steps, occupancy 3), in the pipelined
# (mode 1) and unpipelined (mode 0) schedules.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
COSMOMC_AMD_LIB=$PWD/tools/_d3/libcosmomc_amd.so timeout -k 10 400 python -u -m pytest tests/test_gpu_sampler.py -x -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider -k "pipelined or fused_window or corun" > gpurun_out/r4e_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r4e_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_sampler.py -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "drag" > gpurun_out/r4e_drag_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r4e_drag_tests.log; [ $rc -eq 0 ] || exit $rc
CMAMD_PIPE=1 timeout -k 10 300 python bench.py --steps 100 --no-cpu-baseline --converge-seconds 0 --config4-seconds -1 \
  --config5-seconds -1 --drag-seconds 0 > gpurun_out/r4e_drag.json 2> gpurun_out/r4e_drag.err
rc=$?; [ $rc -eq 0 ] || exit $rc
python -c 'import json; d=json.load(open("gpurun_out/r4e_drag.json"))["config2_drag"]; print("drag", round(d["ms_per_drag_step"]*1e3,1), "us/drag step", d["kernel_us_per_drag_step"])'
run() {   # mode lib tag
  COSMOMC_AMD_LIB=$2 CMAMD_PIPE=$1 timeout -k 10 200 python bench.py --steps 300 --no-cpu-baseline \
    --converge-seconds 0 --config4-seconds -1 --config5-seconds -1 --drag-seconds -1 > gpurun_out/r4e_$3.json 2> gpurun_out/r4e_$3.err
  rc=$?; [ $rc -eq 0 ] || { echo "$3 rc=$rc"; tail -5 gpurun_out/r4e_$3.err; return $rc; }
  python - "$3" <<'PY'
import json, sys
d = json.load(open(f"gpurun_out/r4e_{sys.argv[1]}.json"))
print(sys.argv[1], round(d["value"] / 1e6, 3), "M evals/s", round(d["ms_per_step"] * 1e3, 2), "us/step",
      {k: round(v, 2) for k, v in d["roofline"]["avg_kernel_us"].items() if v})
PY
}
D3=$PWD/tools/_d3/libcosmomc_amd.so; D2O2=$PWD/tools/_d2o2/libcosmomc_amd.so; NT=$PWD/tools/_nt/libcosmomc_amd.so
run 1 "" m1 && run 1 $D3 m1_d3 && run 1 $NT m1_nt && run 1 $D2O2 m1_d2o2 && run 0 "" m0 && run 0 $D3 m0_d3 && \
run 0 $NT m0_nt && run 1 "" m1b && run 1 $D3 m1_d3b && run 1 $NT m1_ntb
