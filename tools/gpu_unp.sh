set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_unproject_gpu.py -q -m gpu -x > gpurun_out/t_unp.log 2>&1 && \
timeout -k 10 120 python tools/bench_unproject.py 32 high > gpurun_out/bu.log 2>&1 && \
timeout -k 10 120 python tools/bench_unproject.py 32 medium >> gpurun_out/bu.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_unp -o unp --output-format csv -- python tools/bench_unproject.py 32 high > gpurun_out/prof_unp.log 2>&1
