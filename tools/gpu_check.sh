#!/bin/bash
# GPU-box session: parity tests, then the bench, then a rocprofv3 kernel
# trace of the bench.  Every GPU step has its own time limit; a crash, abort
# or timeout (anything other than a clean pass/fail) stops the session.
set -u
mkdir -p gpurun_out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/gpu_tests.log
ok $rc || exit $rc
timeout -k 10 300 python bench.py "$@" > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err
[ $rc -eq 0 ] || exit $rc
if [ "${PROFILE:-1}" = "1" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run \
      -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline --converge-seconds 0 --config4-seconds -1 --config5-seconds -1 --drag-seconds -1 "$@" > "$GRAFT_REPO_ROOT/gpurun_out/prof_bench.log" 2>&1
  rc=$?; echo "rocprof rc=$rc"; cd "$GRAFT_REPO_ROOT"
  find gpurun_out/prof -name "*stats*" | head
fi
