# A/B of one dataset's loglike_batch kernels (tools/cmbl_profile.py) with
# alternative library builds (COSMOMC_AMD_LIB): gpu_ab_ds.sh <dataset> <variant>...
set -u
mkdir -p gpurun_out
ds=$1; shift
for v in base "$@"; do
  if [ "$v" = base ]; then unset COSMOMC_AMD_LIB; else export COSMOMC_AMD_LIB=$PWD/tools/$v/libcosmomc_amd.so; fi
  echo "== $v"
  timeout -k 10 120 python -u tools/cmbl_profile.py $ds 1024 30 2>&1 | grep -v amdgpu.ids || exit $?
done
