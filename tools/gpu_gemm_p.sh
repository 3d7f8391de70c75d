# Persistent GEMM engine: bit-exact cross-check vs the tile kernel, kernel tests, microbench A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_engines_gpu.py tests/test_kernels_gpu.py -v -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/t_gemm_p.log 2>&1 || { echo tests_failed; tail -30 gpurun_out/t_gemm_p.log; exit 1; }
rm -f gpurun_out/gemm_ab.log
for P in 0 2 1; do
  I2PC_GEMM_P=$P timeout -k 10 300 python tools/bench_gemm.py >> gpurun_out/gemm_ab.log 2>&1 || { echo bench_failed_$P; tail -5 gpurun_out/gemm_ab.log; exit 1; }
done
echo all_ok
