# DA-v2: per-call GEMM census and in-process A/B of the 384x192 one-round tiles against the alternatives
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/gpu.sh census --model depth-anything-v2 --top 30 || exit 1
bash tools/gpu.sh ab-pipe --model depth-anything-v2 --rounds 4 --variant base: --variant no192:gemm_tile192=0 --variant nobn128:gemm_bn128=0 --variant nostag:gemm_stagger=0 || exit 1
