set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_sampler.py tests/test_gpu_checkpoint.py tests/test_gpu_importance.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_sampler_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/gpu_sampler_tests.log; exit $rc
