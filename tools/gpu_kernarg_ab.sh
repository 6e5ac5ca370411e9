set -u
mkdir -p gpurun_out/karg
export PYTHONUNBUFFERED=1
for v in 0 1 0 1; do
  HIP_FORCE_DEV_KERNARG=$v timeout -k 10 120 python3 bench.py --steps 300 --warmup 20 --no-cpu-baseline --converge-seconds 0 --config4-seconds -1 --config5-seconds -1 --drag-seconds -1 > gpurun_out/karg/b$v.json 2> gpurun_out/karg/b$v.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/karg/b$v.json'));print('KARG=$v', round(d['value']/1e6,3),'M', round(d['ms_per_step']*1e3,2),'us', {k:round(x,2) for k,x in d['roofline']['avg_kernel_us'].items()})"
done
