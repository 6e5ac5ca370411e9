#!/bin/bash
# GPU-box evidence run: the whole -m gpu suite, smoke(), the driver's own bench
# command, the default bench (every leg), a rocprofv3 kernel-trace --stats of
# the headline leg, and the stamp timelines.  Each GPU step has its own limit;
# any failure ends the session.
set -u
TAG=${TAG:-r05}
mkdir -p gpurun_out/$TAG
export PYTHONUNBUFFERED=1
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/$TAG/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/$TAG/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" 2>&1 | grep -v amdgpu.ids; rc=${PIPESTATUS[0]}; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/$TAG/bench_driver.json 2> gpurun_out/$TAG/bench_driver.err; rc=$?; echo "driver-cmd bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 -c "import json;d=json.load(open('gpurun_out/$TAG/bench_driver.json'));print(round(d['value']/1e6,3),'M',round(d['ms_per_step']*1e3,2),'us/step',d['roofline']['kernel'],round(d['roofline']['frac'],3),d['roofline']['avg_kernel_us'])"
timeout -k 10 300 python3 bench.py --steps 500 --no-cpu-baseline --cache-steps -1 --converge-seconds 0 --config1-seconds -1 --config4-seconds -1 --config5-seconds -1 --drag-seconds -1 > gpurun_out/$TAG/bench_500.json 2>/dev/null; rc=$?; [ $rc -eq 0 ] || exit $rc
python3 -c "import json;d=json.load(open('gpurun_out/$TAG/bench_500.json'));print('500 steps:',round(d['value']/1e6,3),'M',round(d['ms_per_step']*1e3,2),'us/step',round(d['roofline']['frac'],3))"
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/$TAG/prof" -o run \
  -- python3 "$R/bench.py" --no-cpu-baseline --cache-steps -1 --converge-seconds 0 --config1-seconds -1 --config4-seconds -1 --config5-seconds -1 --drag-seconds -1 \
  > "$R/gpurun_out/$TAG/prof.log" 2>&1
rc=$?; echo "prof rc=$rc"; rm -f "$R"/gpurun_out/$TAG/prof/*kernel_trace.csv; [ $rc -eq 0 ] || exit $rc
cd "$R"
STAMP_OUT=$PWD/tools/_stamped timeout -k 10 120 python3 tools/uni_stamps.py --no-build 2>&1 | grep -v amdgpu.ids > gpurun_out/$TAG/uni_stamps.txt; cat gpurun_out/$TAG/uni_stamps.txt
STAMP_OUT=$PWD/tools/_stamped timeout -k 10 120 python3 tools/mh_stamps.py --no-build 2>&1 | grep -v amdgpu.ids > gpurun_out/$TAG/mh_stamps.txt; cat gpurun_out/$TAG/mh_stamps.txt
