set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_depth_anything_gpu.py tests/test_kernels_gpu.py tests/test_dpt_gpu.py -q -m gpu -x > gpurun_out/t_da.log 2>&1 || { echo tests_failed; tail -30 gpurun_out/t_da.log; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke_failed; exit 1; }
echo all_ok
