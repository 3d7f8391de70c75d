set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_unproject_gpu.py tests/test_preview_gpu.py -q -m gpu -x > gpurun_out/t_unp.log 2>&1 || { echo tests_failed; tail -30 gpurun_out/t_unp.log; exit 1; }
for P in 1024 2048 4096 8192; do
  I2PC_UNP_PTS=$P timeout -k 10 120 python tools/bench_unproject.py 32 high >> gpurun_out/bu2.log 2>&1 || exit 1
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_unp2 -o unp --output-format csv -- python tools/bench_unproject.py 32 high > gpurun_out/prof_unp2.log 2>&1
echo all_ok
