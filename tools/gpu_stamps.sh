set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 120 python tools/mh_stamps.py --no-build > gpurun_out/mh_stamps.txt 2>&1; rc=$?; cat gpurun_out/mh_stamps.txt | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/tp_stamps.py --no-build > gpurun_out/tp_stamps.txt 2>&1; rc=$?; head -20 gpurun_out/tp_stamps.txt | grep -v amdgpu.ids; exit $rc
