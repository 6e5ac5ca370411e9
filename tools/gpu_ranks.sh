#!/bin/bash
# GPU-box session: bench.py --gpus N as a plain process (it starts the N ranks
# itself), rehearsed with gloo on the one-GPU lease; then the 1-GPU bench.
# Every GPU step has its own time limit; the first failure ends the session.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
N=${N:-2}
timeout -k 10 400 python bench.py --gpus "$N" --dist-backend gloo --steps 200 --no-cpu-baseline \
    --converge-seconds 10 --config4-seconds 10 --config5-seconds 15 --drag-seconds 10 \
    > gpurun_out/bench_g${N}_gloo.json 2> gpurun_out/bench_g${N}_gloo.err
rc=$?; echo "bench --gpus $N rc=$rc"; cat gpurun_out/bench_g${N}_gloo.json; tail -3 gpurun_out/bench_g${N}_gloo.err
[ $rc -eq 0 ] || exit $rc
if [ "${BENCH1:-1}" = "1" ]; then
  timeout -k 10 400 python bench.py > gpurun_out/bench_g1.json 2> gpurun_out/bench_g1.err
  rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_g1.json; tail -3 gpurun_out/bench_g1.err
  [ $rc -eq 0 ] || exit $rc
fi
