#!/bin/bash
# fused-pass item length (CMAMD_TP_MAXL builds in tools/_tpL) against the default 288
set -u
mkdir -p gpurun_out
ARGS="--no-cpu-baseline --steps 300 --warmup 20 --converge-seconds 0 --config4-seconds -1 --config5-seconds -1 --drag-seconds -1"
for L in 288 256 320 384; do
  lib=$PWD/cosmomc_amd/lib/libcosmomc_amd.so; [ $L = 288 ] || lib=$PWD/tools/_tp$L/libcosmomc_amd.so
  COSMOMC_AMD_LIB=$lib timeout -k 10 300 python bench.py $ARGS > gpurun_out/tpl_$L.json 2> gpurun_out/tpl_$L.err || { tail -5 gpurun_out/tpl_$L.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/tpl_$L.json').read().strip().splitlines()[-1])
print('L=$L', round(d['value']/1e6,3), 'M', round(d['ms_per_step']*1e3,2), 'us/step', d['roofline']['avg_kernel_us'])"
done
