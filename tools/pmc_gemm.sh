#!/bin/bash
# PMC passes for one GEMM shape: tools/pmc_gemm.sh <tag> <tile> [m n k]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tag=$1; tile=$2; shift 2
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
           "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum" "FETCH_SIZE"; do
  i=$((i+1))
  I2PC_GEMM_TILE=$tile timeout -k 10 240 rocprofv3 --pmc $grp --kernel-trace -d gpurun_out/pmc_$tag -o p$i --output-format csv -- python tools/gemm_one.py "$@" > gpurun_out/pmc_${tag}_$i.log 2>&1 || exit 1
done
