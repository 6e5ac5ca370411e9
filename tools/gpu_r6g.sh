#!/bin/bash
# Round 6 extra evidence (after tools/gpu_r6e.sh with the same TAG): the PMC
# passes of the configs[1] leg and a two-rank gloo rehearsal of the N > 1 path
# on the one GPU.
set -u
export TAG=${TAG:-r06g}
mkdir -p gpurun_out/$TAG
PMC_OUT=${TAG}_pmc_c1 PMC_BENCH_ARGS="--no-cpu-baseline --steps 5 --warmup 2 --cache-steps -1 --converge-seconds 0 --config1-seconds 3 --config4-seconds -1 --config5-seconds -1 --drag-seconds -1" \
  tools/gpu_pmc.sh || exit $?
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus 2 --steps 20 --warmup 5 --dist-backend gloo --no-cpu-baseline --cache-steps -1 --config1-seconds -1 \
  --config4-seconds -1 --config5-seconds -1 --drag-seconds -1 > gpurun_out/$TAG/g2_gloo.json 2> gpurun_out/$TAG/g2_gloo.err
rc=$?; echo "gloo 2-rank rc=$rc"; tail -c 600 gpurun_out/$TAG/g2_gloo.json; exit $rc
