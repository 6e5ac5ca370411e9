set -u
mkdir -p gpurun_out/hl
export PYTHONUNBUFFERED=1
for v in 8 10 12; do
  if [ $v = 8 ]; then unset COSMOMC_AMD_LIB; else export COSMOMC_AMD_LIB=$PWD/tools/_hl$v/libcosmomc_amd.so; fi
  echo "== COS2 1e-$v"
  timeout -k 10 300 python3 -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_cmblikes.py -k "hl_every or golden or walker_order or walker_counts" -p no:cacheprovider 2>&1 | tail -2
  timeout -k 10 120 python3 tools/hl_margin.py 2>&1 | grep -v amdgpu.ids | tail -9
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --converge-seconds 0 --config1-seconds -1 --config4-seconds -1 --config5-seconds 0 --drag-seconds -1 > gpurun_out/hl/b$v.json 2>/dev/null && python3 -c "import json;d=json.load(open('gpurun_out/hl/b$v.json'));c=d['config5_bk15_plik'];print('config5', round(c['ms_per_step']*1e3,1),'us/step', c['avg_kernel_us'])"
done
