set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rm -f gpurun_out/gemm_ab.log
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -m gpu -x > gpurun_out/t_k.log 2>&1 || { echo tests_failed; tail -30 gpurun_out/t_k.log; exit 1; }
for T in ${TILES:-0 256}; do
  I2PC_GEMM_TILE=$T timeout -k 10 300 python tools/bench_gemm.py >> gpurun_out/gemm_ab.log 2>&1 || { echo bench_failed_$T; exit 1; }
done
echo all_ok
