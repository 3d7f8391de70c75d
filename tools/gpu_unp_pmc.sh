# Unprojection: microbench + kernel trace (VGPR/LDS per dispatch) + PMC passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 python tools/bench_unproject.py 32 high > gpurun_out/unp_bench.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/unp_trace -o run --output-format csv -- python tools/bench_unproject.py 32 high > gpurun_out/unp_trace.log 2>&1 || exit 1
UNP_PTS=${UNP_PTS:-8192} bash tools/pmc_unp.sh || exit 1
echo all_ok
