# A/B: headline bench with environment switches ("NAME=VALUE" arguments)
set -u
mkdir -p gpurun_out
for v in base "$@"; do
  if [ "$v" = base ]; then envs=""; else envs="$v"; fi
  env $envs timeout -k 10 300 python bench.py --steps 300 --no-cpu-baseline --converge-seconds 0 --config5-seconds -1 > gpurun_out/abe.json 2> gpurun_out/abe.err || exit $?
  python -c "import json; d=json.load(open('gpurun_out/abe.json')); print('$v', round(d['value']/1e6,3), {k: round(v, 2) for k, v in d['roofline']['avg_kernel_us'].items() if v})"
done
