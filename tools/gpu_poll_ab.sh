set -u
V1="base"
V2="COSMOMC_AMD_LIB=tools/_x1/libcosmomc_amd.so"
V3="COSMOMC_AMD_LIB=tools/_x2/libcosmomc_amd.so"
V4="COSMOMC_AMD_LIB=tools/_x3/libcosmomc_amd.so"
V5="COSMOMC_AMD_LIB=tools/_x4/libcosmomc_amd.so"
echo "== 300 steps"; REPS=2 bash tools/gpu_ab_env.sh "$V1" "$V2" "$V3" "$V4" "$V5" || exit 1
echo "== 20 steps"; REPS=2 BENCH_ARGS="--steps 20 --warmup 5 --no-cpu-baseline --converge-seconds 0 --config1-seconds -1 --config4-seconds -1 --config5-seconds -1 --drag-seconds -1" bash tools/gpu_ab_env.sh "$V1" "$V2" "$V3" "$V4" "$V5"
