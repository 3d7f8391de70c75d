#!/bin/bash
# Full verification + profile refresh: the -m gpu suite, then C2 and C5 (batch 64) profiles
# (rocprof stats, PMC traffic, bench lines; tools/gpu_profile.sh).
set -o pipefail
bash tools/gpu_check.sh || exit $?
bash tools/gpu_profile.sh dpt-large-bf16 && bash tools/gpu_profile.sh dpt-hybrid-fp8 --model dpt-hybrid --batch 64
