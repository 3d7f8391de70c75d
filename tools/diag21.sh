# sweep range atomics skipped when a relaxed read already covers them: unprojection tests, C4 band
# call trace, C2 / 512 / medium unprojection traces
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_unproject_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t21.log 2>&1 || { tail -20 gpurun_out/t21.log; exit 1; }
tail -1 gpurun_out/t21.log
bash tools/gpu.sh trace-c4 --graph || exit 1
TAG=_c2 bash tools/gpu.sh trace-unp 32 high || exit 1
TAG=_512 bash tools/gpu.sh trace-unp 32 high 512 512 384 384 || exit 1
TAG=_med bash tools/gpu.sh trace-unp 32 medium || exit 1
