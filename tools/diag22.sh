# sweep: range reduced per workgroup, reduction slots re-laid (spike counts off below[2]); tests
# on the stress maps (spike + nanmedian window cases), C4 band call and C2 / 512 / medium traces
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_unproject_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t22.log 2>&1 || { tail -30 gpurun_out/t22.log; exit 1; }
tail -1 gpurun_out/t22.log
bash tools/gpu.sh trace-c4 --graph || exit 1
TAG=_c2 bash tools/gpu.sh trace-unp 32 high || exit 1
TAG=_512 bash tools/gpu.sh trace-unp 32 high 512 512 384 384 || exit 1
TAG=_med bash tools/gpu.sh trace-unp 32 medium || exit 1
