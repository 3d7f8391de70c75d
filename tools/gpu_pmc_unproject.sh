set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/pmc_unp; rm -rf $D; mkdir -p $D
timeout -k 10 120 python tools/bench_unproject.py 32 > $D/bench.txt 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --kernel-trace -d $D/p1 -o p1 --output-format csv -- python tools/bench_unproject.py 32 > $D/p1.txt 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS --kernel-trace -d $D/p2 -o p2 --output-format csv -- python tools/bench_unproject.py 32 > $D/p2.txt 2>&1 || exit 1
python tools/pmc_summary.py $D/p1 unproj:: > $D/s1.txt && python tools/pmc_summary.py $D/p2 unproj:: > $D/s2.txt
cat $D/bench.txt
