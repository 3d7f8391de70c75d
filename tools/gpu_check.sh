#!/bin/bash
# One GPU verification pass: the -m gpu suite (achieved parity errors logged), then a 1-GPU bench.
#   gpurun --timeout 1200 -- bash tools/gpu_check.sh [pytest -k expr]
set -o pipefail
mkdir -p gpurun_out
export I2PC_PARITY_LOG=gpurun_out/parity.jsonl
rm -f "$I2PC_PARITY_LOG"
K=${1:+-k "$1"}
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=5 --timeout 300 --timeout-method thread -rP $K \
  > gpurun_out/gputests.log 2>&1
rc=$?
tail -5 gpurun_out/gputests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err
rc2=$?
cat gpurun_out/bench.json | cut -c1-400
exit $(( rc > rc2 ? rc : rc2 ))
