#!/bin/bash
# Round evidence: the whole -m gpu suite, smoke(), the default bench (every
# leg, CPU baseline included), and a rocprofv3 kernel-trace --stats of the
# headline leg.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" 2>&1 | grep -v amdgpu.ids
rc=$?; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err
rc=$?; echo "bench rc=$rc"; tail -c 400 gpurun_out/bench_full.json; echo
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/final_prof" -o run \
  -- python3 "$R/bench.py" --no-cpu-baseline --converge-seconds 0 --config4-seconds -1 --config5-seconds -1 --drag-seconds -1 \
  > "$R/gpurun_out/final_prof.log" 2>&1
rc=$?; echo "prof rc=$rc"; rm -f "$R"/gpurun_out/final_prof/*kernel_trace.csv; exit $rc
