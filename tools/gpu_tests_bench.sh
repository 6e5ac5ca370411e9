set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/gpu_tests.log | head -20; exit $rc; }
timeout -k 10 200 python bench.py --no-cpu-baseline --converge-seconds 0 --config4-seconds -1 --config5-seconds -1 --drag-seconds -1 > gpurun_out/b.json
rc=$?; [ $rc -eq 0 ] || exit $rc
python3 -c 'import json; d=json.loads(open("gpurun_out/b.json").read().strip().splitlines()[-1]); print(round(d["value"]/1e6,3), "M/s", round(d["ms_per_step"]*1e3,2), "us/step", d["roofline"]["kernel"], round(d["roofline"]["frac"],3), {k: round(v,2) for k,v in d["roofline"]["avg_kernel_us"].items()})'
