# DA-v2 and C5 profiles re-run so their bench lines cite the r04 PMC traffic tables
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out profiles
export ROUND=r04
bash tools/gpu.sh profile depth-anything-v2-small-bf16 --model depth-anything-v2 || exit 1
bash tools/gpu.sh profile dpt-hybrid-fp8 --model dpt-hybrid --batch 64 || exit 1
