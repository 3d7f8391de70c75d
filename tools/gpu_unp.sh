#!/bin/bash
# Unprojection check: GPU parity tests of the geometry path, then the microbench and its
# kernel stats with the row-sweep kernel on and off (I2PC_UNP_ROWS), then the 1-GPU bench.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 400 python -u -m pytest tests/test_unproject_gpu.py tests/test_app_gpu.py tests/test_preview_gpu.py -x -q \
  --timeout 200 --timeout-method thread > gpurun_out/unp_tests.log 2>&1
rc=$?; tail -5 gpurun_out/unp_tests.log; [ $rc -eq 0 ] || exit $rc
for R in 1 0; do
  I2PC_UNP_ROWS=$R timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/unp_prof_$R -o run --output-format csv -- \
    python tools/bench_unproject.py 32 high > gpurun_out/unp_micro_$R.txt 2>&1 || exit 1
  cat gpurun_out/unp_micro_$R.txt | grep B=
  grep -h "k_unproject\|k_sweep<0\|k_resolve<0" $(find gpurun_out/unp_prof_$R -name '*kernel_stats.csv') | cut -c1-160
done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?
cut -c1-300 gpurun_out/bench.json; python -c "
import json; d=json.loads(open('gpurun_out/bench.json').read().strip().splitlines()[-1]); r=d['rooflines']; print('unproject_kernel', r['unproject_kernel']); print('stage', r['unproject_stage'])"
exit $rc
