#!/bin/bash
# Round 6: GPU tests of the changed paths, then an interleaved A/B of the
# unified launch's chi^2 placement (folded into the Metropolis workgroups or
# rows of its own) and the role order, then the binned-cache leg.
set -u
mkdir -p gpurun_out/r6a
export PYTHONUNBUFFERED=1
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_smica.py tests/test_gpu_sampler.py tests/test_gpu_cmblikes.py \
  tests/test_gpu_plik.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r6a/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/r6a/tests.log; [ $rc -eq 0 ] || exit $rc
REPS=2 tools/gpu_ab_env.sh "CMAMD_FOLD_G=0" "base" "CMAMD_TAIL_ORDER=qmp" "CMAMD_TAIL_ORDER=mqp" || exit $?
timeout -k 10 300 python3 bench.py --steps 300 --cache-steps 300 --no-cpu-baseline --converge-seconds 0 \
  --config1-seconds -1 --config4-seconds -1 --config5-seconds -1 --drag-seconds -1 > gpurun_out/r6a/cache.json 2>gpurun_out/r6a/cache.err
rc=$?; echo "cache bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 -c "import json;d=json.loads(open('gpurun_out/r6a/cache.json').read().strip().splitlines()[-1]);print(round(d['value']/1e6,3),'M',round(d['ms_per_step']*1e3,2),'us/step');print(json.dumps(d.get('binned_cache')))"
