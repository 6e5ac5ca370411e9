#!/bin/bash
# Round 6 evidence run: the whole GPU suite, smoke(), the driver's own bench
# command (twice), the 500-step headline, rocprofv3 kernel stats of the
# headline leg, the block timelines and the headline PMC passes.
set -u
TAG=${TAG:-r06e}
mkdir -p gpurun_out/$TAG
export PYTHONUNBUFFERED=1
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/$TAG/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/$TAG/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/$TAG/smoke.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/$TAG/bench_driver$i.json 2> gpurun_out/$TAG/bench_driver$i.err; rc=$?; echo "driver-cmd bench $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 -c "import json;d=json.load(open('gpurun_out/$TAG/bench_driver$i.json'));print(round(d['value']/1e6,3),'M',round(d['ms_per_step']*1e3,2),'us/step',d['roofline']['kernel'],round(d['roofline']['frac'],3),d['roofline']['avg_kernel_us']);print({k:(round(v['ms_per_step']*1e3,2) if 'ms_per_step' in v else round(v.get('ms_per_drag_step',0)*1e3,2)) for k,v in d.items() if k.startswith('config') and isinstance(v,dict) and ('ms_per_step' in v or 'ms_per_drag_step' in v)}); print('cache', d.get('binned_cache',{}).get('ms_per_step'), d.get('binned_cache',{}).get('step_roofline',{}).get('frac'))"
done
timeout -k 10 300 python3 bench.py --steps 500 --no-cpu-baseline --cache-steps -1 --converge-seconds 0 --config1-seconds -1 --config4-seconds -1 --config5-seconds -1 --drag-seconds -1 > gpurun_out/$TAG/bench_500.json 2>/dev/null; rc=$?; [ $rc -eq 0 ] || exit $rc
python3 -c "import json;d=json.load(open('gpurun_out/$TAG/bench_500.json'));print('500 steps:',round(d['value']/1e6,3),'M',round(d['ms_per_step']*1e3,2),'us/step',round(d['roofline']['frac'],3))"
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/$TAG/prof" -o run \
  -- python3 "$R/bench.py" --no-cpu-baseline --cache-steps -1 --converge-seconds 0 --config1-seconds -1 --config4-seconds -1 --config5-seconds -1 --drag-seconds -1 \
  > "$R/gpurun_out/$TAG/prof.log" 2>&1
rc=$?; echo "prof rc=$rc"; rm -f "$R"/gpurun_out/$TAG/prof/*kernel_trace.csv; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/$TAG/prof_driver" -o run \
  -- python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --converge-seconds 0 --config1-seconds -1 --config4-seconds -1 --config5-seconds -1 --drag-seconds -1 \
  > "$R/gpurun_out/$TAG/prof_driver.log" 2>&1
rc=$?; echo "prof driver rc=$rc"; rm -f "$R"/gpurun_out/$TAG/prof_driver/*kernel_trace.csv; [ $rc -eq 0 ] || exit $rc
cd "$R"
STAMP_OUT=$PWD/tools/_stamped timeout -k 10 120 python3 tools/uni_stamps.py --no-build > gpurun_out/$TAG/uni_stamps.txt 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/$TAG/uni_stamps.txt; [ $rc -eq 0 ] || exit $rc
PMC_OUT=${TAG}_pmc tools/gpu_pmc.sh
