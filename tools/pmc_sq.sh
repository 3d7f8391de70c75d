# SQ counter passes (one group per rocprofv3 run, kernel-trace only) over the attention and GEMM
# microbenchmarks: where the waves of the two dominant network kernels spend their cycles.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rm -rf gpurun_out/pmc_sq
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  for prog in bench_attn bench_gemm; do
    timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace -d gpurun_out/pmc_sq -o ${prog}_$i --output-format csv -- python tools/$prog.py > gpurun_out/pmc_sq_${prog}_$i.txt 2>&1 || { echo "pmc pass $i $prog failed"; tail -5 gpurun_out/pmc_sq_${prog}_$i.txt; exit 1; }
  done
done
python tools/pmc_summary.py gpurun_out/pmc_sq k_attention > gpurun_out/pmc_sq_attn.txt
python tools/pmc_summary.py gpurun_out/pmc_sq k_gemm_p > gpurun_out/pmc_sq_gemm.txt
echo all_ok
