#!/bin/bash
# Round 6: the folded chi^2's latency (stamps), A/B of its tasks in flight,
# the quadratic form's priority, the role order and the unfolded chi^2, and the
# configs[4] leg with the decorrelation-free window group kernel.
set -u
mkdir -p gpurun_out/r6f
export PYTHONUNBUFFERED=1
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_sampler.py tests/test_gpu_cmblikes.py tests/test_gpu_smica.py -m gpu -x -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r6f/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r6f/tests.log; [ $rc -eq 0 ] || exit $rc
for v in "" "CMAMD_FOLD_TPF=2"; do
  env $v STAMP_OUT=$PWD/tools/_stamped timeout -k 10 120 python3 tools/uni_stamps.py --no-build > gpurun_out/r6f/stamps.txt 2>&1
  rc=$?; echo "== stamps [$v]"; grep -v amdgpu.ids gpurun_out/r6f/stamps.txt | head -7; [ $rc -eq 0 ] || exit $rc
done
REPS=2 tools/gpu_ab_env.sh "base" "CMAMD_FOLD_TPF=2" "CMAMD_QF_PRIO=1" "CMAMD_TAIL_ORDER=qmp" "CMAMD_FOLD_G=0" || exit $?
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --cache-steps -1 --converge-seconds 0 --config1-seconds -1 \
  --config4-seconds -1 --config5-seconds 0 --drag-seconds -1 > gpurun_out/r6f/c5.json 2>/dev/null; rc=$?; [ $rc -eq 0 ] || exit $rc
python3 -c "import json;d=json.loads(open('gpurun_out/r6f/c5.json').read().strip().splitlines()[-1]);c=d['config5_bk15_plik'];print('config5',round(c['ms_per_step']*1e3,2),c['avg_kernel_us'])"
