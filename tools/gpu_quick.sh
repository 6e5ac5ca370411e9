#!/bin/bash
# Quick GPU check: the schedule / hand-off tests, the driver's bench command, the unified launch's stamps
set -u
TAG=${TAG:-quick}
mkdir -p gpurun_out/$TAG
export PYTHONUNBUFFERED=1
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_sampler.py -k "${KSEL:-pipelined or handoff or plik_fast_chain or bin_corun or config5_joint}" > gpurun_out/$TAG/tests.log 2>&1; rc=$?; tail -2 gpurun_out/$TAG/tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --converge-seconds 0 --config1-seconds -1 --config4-seconds -1 --config5-seconds -1 --drag-seconds -1 > gpurun_out/$TAG/bench20.json 2>/dev/null; rc=$?; [ $rc -eq 0 ] || exit $rc
python3 -c "import json;d=json.load(open('gpurun_out/$TAG/bench20.json'));print('20 steps:',round(d['value']/1e6,3),'M',round(d['ms_per_step']*1e3,2),'us/step',{k:round(v,2) for k,v in d['roofline']['avg_kernel_us'].items()})"
done
timeout -k 10 300 python3 bench.py --steps 500 --no-cpu-baseline --converge-seconds 0 --config1-seconds -1 --config4-seconds -1 --config5-seconds -1 --drag-seconds -1 > gpurun_out/$TAG/bench500.json 2>/dev/null; rc=$?; [ $rc -eq 0 ] || exit $rc
python3 -c "import json;d=json.load(open('gpurun_out/$TAG/bench500.json'));print('500 steps:',round(d['value']/1e6,3),'M',round(d['ms_per_step']*1e3,2),'us/step',{k:round(v,2) for k,v in d['roofline']['avg_kernel_us'].items()})"
STAMP_OUT=$PWD/tools/_stamped timeout -k 10 120 python3 tools/uni_stamps.py --no-build 2>&1 | grep -v amdgpu.ids > gpurun_out/$TAG/uni_stamps.txt; cat gpurun_out/$TAG/uni_stamps.txt
