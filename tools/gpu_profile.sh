#!/bin/bash
# Profiles of one bench configuration, committed under profiles/ (one script for every round):
#   1) rocprofv3 --kernel-trace --stats over the bench command itself (graph-replayed steps)
#      -> profiles/<round>_<tag>_kernel_stats.csv and the bench line -> profiles/<round>_<tag>_bench.json
#   2) two --pmc passes (FETCH_SIZE, WRITE_SIZE; kernel-trace only, separate runs) over one
#      eager step -> profiles/<round>_<tag>_pmc_traffic.json (tools/pmc_traffic.py, gfx950 correction)
#   gpurun --timeout 1200 -- bash tools/gpu_profile.sh <tag> [bench args ...]
set -o pipefail
TAG=$1; shift
R=${ROUND:-r02}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/prof_$TAG
rm -rf "$D"; mkdir -p "$D" profiles
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$D/stats" -o run --output-format csv -- \
  python bench.py --steps 10 --warmup 3 --no-cpu-baseline "$@" > "$D/bench.json" 2> "$D/bench.err" \
  || { echo "stats run failed"; tail -5 "$D/bench.err"; exit 1; }
for grp in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace -d "$D/pmc" -o $grp --output-format csv -- \
    python bench.py --steps 1 --warmup 0 --no-graph --no-kernel-profile --no-cpu-baseline "$@" > "$D/pmc_$grp.txt" 2>&1 \
    || { echo "pmc pass $grp failed"; tail -5 "$D/pmc_$grp.txt"; exit 1; }
done
python tools/pmc_traffic.py "$D/pmc" "profiles/${R}_${TAG}_pmc_traffic.json" || exit 1
cp "$(find "$D/stats" -name '*kernel_stats.csv' | head -1)" "profiles/${R}_${TAG}_kernel_stats.csv" || exit 1
tail -1 "$D/bench.json" > "profiles/${R}_${TAG}_bench.json"
cp profiles/${R}_${TAG}_* gpurun_out/
echo profile_ok
