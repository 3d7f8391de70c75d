# round-4 closing bundle: new tests, unprojection rows-per-thread sweep, C4 evidence, full check
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out profiles
export ROUND=r04
timeout -k 10 500 python -u -m pytest tests/test_determinism_gpu.py "tests/test_gemm_engines_gpu.py::test_stagger_bitexact" -x -q --timeout 300 --timeout-method thread > gpurun_out/t20.log 2>&1 || { tail -20 gpurun_out/t20.log; exit 1; }
tail -1 gpurun_out/t20.log
bash tools/diag19.sh || exit 1
bash tools/gpu.sh check || exit 1
