# GPU session: CMBlikes parity (BK grouped window kernel), then BK profiles
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_cmblikes.py -x -q --timeout 200 --timeout-method thread -m gpu -p no:cacheprovider > gpurun_out/g4_tests.log 2>&1
rc=$?; tail -15 gpurun_out/g4_tests.log; [ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/g4_prof.log
for c in bk15 bk; do
  timeout -k 10 120 python -u tools/cmbl_profile.py $c 1024 30 >> gpurun_out/g4_prof.log 2>&1 || exit $?
done
grep -v amdgpu.ids gpurun_out/g4_prof.log
