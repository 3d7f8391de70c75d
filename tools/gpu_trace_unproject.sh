#!/bin/bash
# Per-kernel durations of the geometry-stage microbenchmark (kernel trace only, no counters):
#   gpurun -- bash tools/gpu_trace_unproject.sh [batch] [density]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/trace_unp; rm -rf $D; mkdir -p $D
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $D/t -o t --output-format csv -- \
  python tools/bench_unproject.py ${1:-32} ${2:-high} > $D/bench.txt 2>&1 || { tail -5 $D/bench.txt; exit 1; }
cat $D/bench.txt | tail -1
python - "$D" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/t/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "unproj" in r["Name"]:
        print(f'{float(r["AverageNs"])/1e3:8.1f} us  x{r["Calls"]:>4}  {r["Name"][:70]}')
PY
