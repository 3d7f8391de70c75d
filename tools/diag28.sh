# skinny GEMM off by default: the full GPU suite and the bench
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export ROUND=r04
bash tools/gpu.sh check || exit 1
