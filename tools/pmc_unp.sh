#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, kernel-trace only) over the unprojection microbench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_ACTIVE_INST_VALU" \
           "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  I2PC_UNP_PTS=${UNP_PTS:-8192} timeout -k 10 240 rocprofv3 --pmc $grp --kernel-trace -d gpurun_out/pmc_unp -o p$i --output-format csv -- python tools/bench_unproject.py 32 high > gpurun_out/pmc_unp_$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 gpurun_out/pmc_unp_$i.log; exit 1; }
done
python tools/pmc_summary.py gpurun_out/pmc_unp unproj > gpurun_out/pmc_unp_summary.txt
echo all_ok
