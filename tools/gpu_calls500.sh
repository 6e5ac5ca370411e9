#!/bin/bash
# Kernel trace of a 500-step headline call: per-launch durations over the call
set -u
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/calls500"
mkdir -p "$OUT"
NB="--no-cpu-baseline --converge-seconds 0 --config1-seconds -1 --config4-seconds -1 --config5-seconds -1 --drag-seconds -1"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/tr" -o run \
  -- python3 "$R/bench.py" --gpus 1 --steps 500 --warmup ${WU:-5} $NB > "$OUT/trace_bench.json" 2>/dev/null || exit $?
python3 - "$OUT/tr/run_kernel_trace.csv" <<'PY' | tee "$OUT/calls.txt"
import csv, sys
import numpy as np
rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(open(sys.argv[1]))
              if "mh_step_kernel" in r["Kernel_Name"])
d = np.array([(e - s) * 1e-3 for s, e in rows])
# the timed call is launches [4, 4 + 499) after the warmup's 4 middle launches
for name, seg in (("warmup", d[:4]), ("timed", d[4:503]), ("profiled", d[503:])):
    print(name, len(seg), "mean %.2f" % seg.mean() if len(seg) else "")
    for a in range(0, len(seg), 50):
        print("   steps %3d-%3d mean %.2f min %.2f max %.2f" % (a, min(a + 50, len(seg)), seg[a:a + 50].mean(), seg[a:a + 50].min(), seg[a:a + 50].max()))
PY
rm -f "$OUT"/tr/*.csv
