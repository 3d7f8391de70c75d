#!/bin/bash
# SQ (shader) counters of one eager bench step, two passes of 8 counters, summarised per kernel
# for the attention and the persistent GEMM -> gpurun_out/<round>_<tag>_sq.txt (copy to profiles/):
#   gpurun --timeout 900 -- bash tools/gpu_sq_profile.sh <tag> [bench args ...]
set -o pipefail
TAG=$1; shift
R=${ROUND:-r02}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/sq_$TAG
rm -rf "$D"; mkdir -p "$D"
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"
P2="SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS"
i=0
for grp in "$P1" "$P2"; do
  i=$((i + 1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace -d "$D/p$i" -o p$i --output-format csv -- \
    python bench.py --steps 1 --warmup 0 --no-graph --no-kernel-profile --no-cpu-baseline "$@" > "$D/p$i.txt" 2>&1 \
    || { echo "pass $i failed"; tail -5 "$D/p$i.txt"; exit 1; }
done
{ for f in attention gemm_p; do python tools/pmc_summary.py "$D/p1" $f; python tools/pmc_summary.py "$D/p2" $f; done; } \
  > "gpurun_out/${R}_${TAG}_sq.txt" || exit 1
echo sq_ok
