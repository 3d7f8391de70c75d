set -o pipefail
cd $GRAFT_REPO_ROOT
for t in 256 8; do bash tools/pmc_gemm.sh t$t $t 18464 3072 1024 || { echo fail_$t; exit 1; }; python tools/pmc_summary.py gpurun_out/pmc_t$t gemm > gpurun_out/pmc_t${t}_summary.txt; done
echo all_ok
