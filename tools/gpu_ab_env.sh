#!/bin/bash
# Interleaved A/B of the headline bench under environment switches.
#   tools/gpu_ab_env.sh "base" "CMAMD_PIPE=0" "CMAMD_UNI_WT=8" ...
# Each argument is one variant ("base": no extra environment); REPS (default 2)
# rounds run every variant in turn; BENCH_ARGS replaces the default bench
# arguments (headline only, 300 steps).
set -u
mkdir -p gpurun_out/ab
REPS=${REPS:-2}
ARGS=${BENCH_ARGS:---steps 300 --warmup 20 --no-cpu-baseline --cache-steps -1 --converge-seconds 0 --config1-seconds -1 --config4-seconds -1 --config5-seconds -1 --drag-seconds -1}
for rep in $(seq 1 $REPS); do
  i=0
  for v in "$@"; do
    i=$((i + 1))
    if [ "$v" = base ]; then envs=""; else envs="$v"; fi
    env $envs timeout -k 10 300 python3 bench.py $ARGS > gpurun_out/ab/v${i}_$rep.json 2> gpurun_out/ab/v${i}_$rep.err || exit $?
    python3 - "$v" "$rep" gpurun_out/ab/v${i}_$rep.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
print(f"[{sys.argv[1]}] rep {sys.argv[2]}: {d['value'] / 1e6:.3f} M evals/s {d['ms_per_step'] * 1e3:.2f} us/step",
      {k: round(v, 2) for k, v in d["roofline"]["avg_kernel_us"].items() if v}, flush=True)
for leg in ("config1_tt", "config4_fast21", "config5_bk15_plik", "config2_drag"):
    c = d.get(leg)
    if isinstance(c, dict) and ("ms_per_step" in c or "ms_per_drag_step" in c):
        t = c.get("ms_per_step", c.get("ms_per_drag_step"))
        print(f"    {leg}: {t * 1e3:.2f} us/step", c.get("kernel_us_per_step", c.get("kernel_us_per_drag_step", "")),
              flush=True)
PY
  done
done
