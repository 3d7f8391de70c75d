#!/bin/bash
# Per-kernel durations of the unprojection launches inside the real bench step (kernel trace only):
#   gpurun -- bash tools/gpu_trace_bench.sh [bench args]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/trace_bench; rm -rf $D; mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/t -o t --output-format csv -- \
  python bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > $D/bench.json 2> $D/bench.err || { tail -5 $D/bench.err; exit 1; }
python - "$D" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/t/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "unproj" in r["Name"]:
        print(f'{float(r["AverageNs"])/1e3:8.1f} us  x{r["Calls"]:>4}  {r["Name"][:70]}')
PY
