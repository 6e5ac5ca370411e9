# A/B: headline bench with alternative library builds (COSMOMC_AMD_LIB)
set -u
mkdir -p gpurun_out
for v in base "$@"; do
  if [ "$v" = base ]; then unset COSMOMC_AMD_LIB; else export COSMOMC_AMD_LIB=$PWD/tools/$v/libcosmomc_amd.so; fi
  timeout -k 10 300 python bench.py --steps 300 --no-cpu-baseline --converge-seconds 0 --config5-seconds -1 --config4-seconds -1 --drag-seconds -1 > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || exit $?
  python -c "import json; d=json.load(open('gpurun_out/ab_$v.json')); print('$v', round(d['value']/1e6,3), {k: round(v, 2) for k, v in d['roofline']['avg_kernel_us'].items() if v})"
done
