set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
O=gpurun_out/diag7.txt; rm -f $O
export I2PC_PARITY_LOG=gpurun_out/parity7.jsonl; rm -f $I2PC_PARITY_LOG
timeout -k 10 600 python -u -m pytest tests/test_dpt_gpu.py tests/test_ln_fold_gpu.py tests/test_gemm_engines_gpu.py -x -q -rP --timeout 300 --timeout-method thread > gpurun_out/t7.log 2>&1; rc=$?
grep -h "parity\|passed\|failed\|Error" gpurun_out/t7.log | head -40 >> $O
[ $rc -eq 0 ] || { cat $O; tail -30 gpurun_out/t7.log; exit 1; }
for v in 1 0 1 0; do
  I2PC_BF16_STREAM=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/b7_$v.json 2>/dev/null || exit 1
  echo "stream=$v $(python -c "import json;d=json.loads(open('gpurun_out/b7_$v.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['rooflines']['dpt_blocks']['frac'])")" >> $O
done
grep -v amdgpu.ids $O
