#!/bin/bash
# Unprojection kernel variants (one process each: the knobs are read once): warm / cold
# microbench, then the geometry parity tests and the 1-GPU bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_unproject_gpu.py tests/test_gemm_engines_gpu.py -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/unp_tests.log 2>&1; rc=$?; tail -2 gpurun_out/unp_tests.log; [ $rc -eq 0 ] || exit $rc
for v in "ROWS=1 NT=1 RPT=8" "ROWS=1 NT=0 RPT=8" "ROWS=1 NT=1 RPT=4" "ROWS=1 NT=0 RPT=4" "ROWS=0 NT=1 RPT=8"; do
  set -- $v
  env I2PC_UNP_$1 I2PC_UNP_$2 I2PC_UNP_$3 timeout -k 10 120 python tools/bench_unproject.py 32 high > gpurun_out/v.txt 2>&1 || exit 1
  echo "$v: $(grep -h 'B=' gpurun_out/v.txt | sed 's/algorithmic.*//' | tr '\n' ' ')"
done
I2PC_GEMM_TAIL=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_notail.json 2> gpurun_out/bench.err || exit 1
echo "no tail split: $(cut -c1-200 gpurun_out/bench_notail.json)"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?
python -c "
import json; d=json.loads(open('gpurun_out/bench.json').read().strip().splitlines()[-1]); r=d['rooflines']; print(d['value'], d['ms_per_step']); print('unproject_kernel', r['unproject_kernel']['us'], r['unproject_kernel']['frac']); print('stage', r['unproject_stage']['ms'], r['unproject_stage']['frac'])"
exit $rc
