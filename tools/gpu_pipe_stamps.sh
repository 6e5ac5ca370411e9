set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 120 python tools/pipe_stamps.py --no-build > gpurun_out/pipe_stamps.txt 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/pipe_stamps.txt; exit $rc
