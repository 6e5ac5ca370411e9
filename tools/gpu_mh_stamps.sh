set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 120 python tools/mh_stamps.py --no-build > gpurun_out/mh_stamps.txt 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/mh_stamps.txt; exit $rc
