# GPU session: SPTpol / CMBlikes / importance parity, then per-dataset profiles
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_cmblikes.py tests/test_gpu_sptpol.py tests/test_gpu_importance.py -x -q --timeout 200 --timeout-method thread -m gpu -p no:cacheprovider > gpurun_out/g3_tests.log 2>&1
rc=$?; tail -5 gpurun_out/g3_tests.log; [ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/g3_prof.log
for c in sptteee sptbb bk15 bk; do
  timeout -k 10 120 python -u tools/cmbl_profile.py $c 1024 30 >> gpurun_out/g3_prof.log 2>&1 || exit $?
done
grep -v amdgpu.ids gpurun_out/g3_prof.log
