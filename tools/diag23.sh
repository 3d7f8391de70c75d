# round-4 closing profiles after the sweep fix: C4 modes, C2 / medium / 512 profiles, full check
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out profiles
export ROUND=r04
bash tools/gpu.sh c4 > gpurun_out/c4.txt 2>&1 || { tail -5 gpurun_out/c4.txt; exit 1; }
grep -h '^{' gpurun_out/c4.jsonl | cut -c1-200
bash tools/gpu.sh profile dpt-large-bf16 || exit 1
bash tools/gpu.sh profile dpt-large-bf16-medium --density medium || exit 1
bash tools/gpu.sh profile dpt-large-bf16-512 --size 512 || exit 1
bash tools/gpu.sh check || exit 1
