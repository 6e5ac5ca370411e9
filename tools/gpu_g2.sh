set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_cmblikes.py tests/test_gpu_sptpol.py -x -q --timeout 200 --timeout-method thread -m gpu -p no:cacheprovider > gpurun_out/g2_tests.log 2>&1
rc=$?; tail -5 gpurun_out/g2_tests.log; [ $rc -eq 0 ] || exit $rc
for c in sptteee sptbb bk15 bk lensing; do
  timeout -k 10 120 python -u tools/cmbl_profile.py $c 1024 30 >> gpurun_out/g2_prof.log 2>&1 || exit $?
done
cat gpurun_out/g2_prof.log
