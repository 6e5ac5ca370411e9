#!/bin/bash
# HL kernel: CMBlikes parity, then the BK15 + plik leg (BASELINE configs[4]) throughput
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_cmblikes.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/hl_tests.log 2>&1
rc=$?; tail -3 gpurun_out/hl_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 50 --no-cpu-baseline --converge-seconds 0 --config4-seconds -1 --config5-seconds 0 --drag-seconds -1 > gpurun_out/bench_hl.json 2> gpurun_out/bench_hl.err
rc=$?; python -c "
import json; d=json.load(open('gpurun_out/bench_hl.json')); c=d['config5_bk15_plik']; print('headline', round(d['value']/1e6,3), 'config5', round(c['evals_per_s']/1e6,3), round(c['ms_per_step']*1e3,1), c['avg_kernel_us'])"
exit $rc
