# HBM traffic of the bench's kernels: one rocprofv3 --pmc pass per counter (FETCH_SIZE, then
# WRITE_SIZE; kernel-trace only) over a short eager bench run -> profiles/<round>_pmc_traffic.json.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
R=${ROUND:-r01}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/pmc_bench
i=0
for grp in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace -d gpurun_out/pmc_bench -o p$i --output-format csv -- python bench.py --steps 1 --warmup 0 --no-graph --no-kernel-profile --no-cpu-baseline > gpurun_out/pmc_bench_$i.txt 2>&1 || { echo "pmc pass $i failed"; tail -5 gpurun_out/pmc_bench_$i.txt; exit 1; }
done
python tools/pmc_traffic.py gpurun_out/pmc_bench profiles/${R}_pmc_traffic.json || exit 1
cp profiles/${R}_pmc_traffic.json gpurun_out/ && echo all_ok
