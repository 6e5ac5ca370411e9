# plik GPU parity, then a short headline bench (kernel averages)
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_plik.py tests/test_gpu_cmblikes.py tests/test_gpu_sptpol.py -x -q --timeout 200 --timeout-method thread -m gpu -p no:cacheprovider > gpurun_out/qf.log 2>&1
rc=$?; tail -2 gpurun_out/qf.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 300 --no-cpu-baseline --converge-seconds 0 --config5-seconds -1 > gpurun_out/qf.json 2> gpurun_out/qf.err || exit $?
python -c "import json; d=json.load(open('gpurun_out/qf.json')); print(d['value'], d['roofline']['achieved'], {k: round(v, 2) for k, v in d['roofline']['avg_kernel_us'].items() if v})"
