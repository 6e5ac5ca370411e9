#!/bin/bash
# lean chain + per-problem HL stop: the schedule / determinism tests, an interleaved A/B, stamps
set -u
mkdir -p gpurun_out/lean
export PYTHONUNBUFFERED=1
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_sampler.py tests/test_gpu_cmblikes.py tests/test_gpu_plik.py -k "configs1 or pipelined_steps_bitwise or plik_fast_chain or pipelined_with_wide or handoff_giveup or config5_joint or walker_order or hl_every or golden" > gpurun_out/lean/tests.log 2>&1; rc=$?; tail -3 gpurun_out/lean/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/ab_steps.py --steps 300 --reps 2 > gpurun_out/lean/ab.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/lean/ab.log; [ $rc -eq 0 ] || exit $rc
STAMP_OUT=$PWD/tools/_stamped timeout -k 10 120 python3 tools/mh_stamps.py --no-build > gpurun_out/lean/stamps.txt 2>&1; grep -v amdgpu.ids gpurun_out/lean/stamps.txt
timeout -k 10 120 python3 tools/hl_margin.py > gpurun_out/lean/hl_margin.txt 2>&1; grep -v amdgpu.ids gpurun_out/lean/hl_margin.txt
timeout -k 10 300 python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline --converge-seconds 0 --config1-seconds 0 --config4-seconds -1 --config5-seconds 0 --drag-seconds -1 > gpurun_out/lean/bench.json 2> gpurun_out/lean/bench.err; python3 -c "import json;d=json.load(open('gpurun_out/lean/bench.json'));print(round(d['value']/1e6,3),'M',round(d['ms_per_step']*1e3,2),'us',d['roofline']['avg_kernel_us']);print('config1',{k:v for k,v in d['config1_tt'].items() if 'trace' not in k});print('config5',{k:v for k,v in d['config5_bk15_plik'].items() if 'trace' not in k})"
STAMP_OUT=$PWD/tools/_stamped timeout -k 10 120 python3 tools/uni_stamps.py --no-build > gpurun_out/lean/uni_stamps.txt 2>&1; grep -v amdgpu.ids gpurun_out/lean/uni_stamps.txt | head -12
