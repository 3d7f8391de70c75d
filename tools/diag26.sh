# C2: per-call census (neck GEMM shapes) and in-process A/B of the split-K knobs that pick their tiles
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/gpu.sh census --top 45 || exit 1
bash tools/gpu.sh ab-pipe --rounds 4 --variant base: --variant nosplitk:gemm_splitk=0 --variant splittile:gemm_split_tile=1 || exit 1
