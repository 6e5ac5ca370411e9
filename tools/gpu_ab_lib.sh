# A/B of the in-tree library against tools/_ab/libcosmomc_amd.so (another build), headline bench only
set -u
mkdir -p gpurun_out
for v in new old new old; do
  if [ $v = old ]; then export COSMOMC_AMD_LIB=$PWD/tools/_ab/libcosmomc_amd.so; else unset COSMOMC_AMD_LIB; fi
  timeout -k 10 200 python bench.py --no-cpu-baseline --converge-seconds 0 --config4-seconds -1 --config5-seconds -1 --drag-seconds -1 > gpurun_out/ab_$v.json || exit 1
  python3 -c 'import json,sys; d=json.loads(open("gpurun_out/ab_'$v'.json").read().strip().splitlines()[-1]); print("'$v'", round(d["value"]/1e6,3), "M/s", round(d["ms_per_step"]*1e3,2), "us/step", {k: round(v,2) for k,v in d["roofline"]["avg_kernel_us"].items()})'
done
