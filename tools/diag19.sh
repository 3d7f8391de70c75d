cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out profiles
bash tools/diag18.sh || exit 1
bash tools/gpu.sh trace-c4 --graph > gpurun_out/trace_c4.txt 2>&1 || { tail -5 gpurun_out/trace_c4.txt; exit 1; }
cp "$(find gpurun_out/trace_c4/t -name '*kernel_stats.csv' | head -1)" profiles/r04_c4_band_kernel_stats.csv
cat gpurun_out/trace_c4.txt
bash tools/gpu.sh c4 > gpurun_out/c4.txt 2>&1 || { tail -5 gpurun_out/c4.txt; exit 1; }
cp gpurun_out/c4.jsonl profiles/r04_c4_panorama_1rank.jsonl
cat gpurun_out/c4.txt
