#!/bin/bash
# Round profile refresh: C2 and C5 rocprof stats + PMC traffic (tools/gpu_profile.sh), then the
# default bench line (with the CPU baseline) as the driver runs it.
set -o pipefail
bash tools/gpu_profile.sh dpt-large-bf16 && bash tools/gpu_profile.sh dpt-hybrid-fp8 --model dpt-hybrid || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err; rc=$?
cut -c1-400 gpurun_out/bench_default.json; exit $rc
