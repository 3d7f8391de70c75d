set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -m gpu -x -k attention > gpurun_out/t_attn.log 2>&1 || { echo tests_failed; tail -30 gpurun_out/t_attn.log; exit 1; }
rm -f gpurun_out/attn_ab.log
I2PC_ATTN_OLD=1 timeout -k 10 120 python tools/bench_attn.py >> gpurun_out/attn_ab.log 2>&1 || exit 1
timeout -k 10 120 python tools/bench_attn.py >> gpurun_out/attn_ab.log 2>&1 || exit 1
for T in 8 256; do
  I2PC_GEMM_TILE=$T timeout -k 10 300 python tools/bench_gemm.py >> gpurun_out/gemm_ab.log 2>&1 || { echo bench_failed_$T; exit 1; }
done
echo all_ok
