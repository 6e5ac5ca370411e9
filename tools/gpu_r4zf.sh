#!/bin/bash
# Round 4: HL sweep-stop threshold (cos^2 1e-12 default, 1e-10, 1e-8): golden margins and BK15 timing
set -u
mkdir -p gpurun_out
for v in def 10 8; do
  lib=""; [ "$v" != def ] && lib="$PWD/tools/_hl$v/libcosmomc_amd.so"
  echo "== cos2 $v"
  COSMOMC_AMD_LIB=$lib timeout -k 10 200 python tools/hl_margin.py 2>&1 | grep -v amdgpu.ids | grep -i "bk\|hl\|max rel" | head -12 || exit $?
  COSMOMC_AMD_LIB=$lib timeout -k 10 200 python tools/cmbl_profile.py bk15 1024 20 2>&1 | grep -E "hl_kernel|total" || exit $?
done
