#!/bin/bash
# The round-end checks on the final tree: the GPU suite, smoke() and the
# driver's bench command.
set -u
mkdir -p gpurun_out/final
export PYTHONUNBUFFERED=1
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/final/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/final/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/final/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/final/bench.json 2> gpurun_out/final/bench.err; rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 -c "import json;d=json.load(open('gpurun_out/final/bench.json'));print(round(d['value']/1e6,3),'M',round(d['ms_per_step']*1e3,2),'us/step',round(d['roofline']['frac'],3),d['roofline']['traffic'])"
