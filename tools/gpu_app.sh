set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_preview_gpu.py tests/test_app_gpu.py tests/test_unproject_gpu.py -q -m gpu -x > gpurun_out/t_app.log 2>&1 || { echo tests_failed; tail -40 gpurun_out/t_app.log; exit 1; }
echo all_ok
