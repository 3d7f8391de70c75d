set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_engines_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/eng.log 2>&1
rc=$?; tail -15 gpurun_out/eng.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bench_gemm_ab.py > gpurun_out/ab.log 2>&1; rc=$?; cat gpurun_out/ab.log; exit $rc
