#!/bin/bash
# Every GPU-box task of this repo, one script (run through gpurun):
#   gpurun --timeout 1200 -- bash tools/gpu.sh <task> [args]
# tasks
#   check [pytest -k expr]     the -m gpu suite (achieved parity errors -> gpurun_out/parity.jsonl), then a 1-GPU bench
#   profile <tag> [bench args] rocprofv3 --kernel-trace --stats over the bench + two --pmc passes (FETCH_SIZE,
#                              WRITE_SIZE; kernel trace only) -> profiles/<round>_<tag>_{kernel_stats.csv,
#                              pmc_traffic.json,bench.json}, copied to gpurun_out/ (copy them back to profiles/)
#   sq <tag> [bench args]      SQ counters (two passes of 8) of one eager step for attention and the persistent GEMM
#   full                       check + profile of C2 (dpt-large-bf16) and C5 (dpt-hybrid-fp8, batch 64)
#   final1 / final2            the round's record: check (+ profiles/<round>_bench_check.json) and the C2 high /
#                              medium profiles; the DA-v2 and C5 profiles
#   bench                      the default bench line (with the CPU baseline), as the driver runs it
#   ab-pipe [args]             tools/ab_pipeline.py: kernel-selection knobs A/B on the bench pipeline, one process
#   census [args]              tools/gemm_census.py: every network launch with shape, kernel and rate
#   gm                         census of the C2 network per GEMM tile-order GROUP_M (2, 4, 8, 16)
#   ab-gemm                    GEMM engine tests + tools/bench_gemm_ab.py (engine modes, interleaved)
#   unp                        geometry parity tests, unprojection microbench (warm / cold) per kernel variant
#   trace-unp [B] [density] [H W h w]  kernel durations of the unprojection microbench (kernel trace
#                              only; TAG=<suffix> names the output directory)
#   pmc-unp                    SQ counters of the unprojection microbench
#   c4                         tools/c4_panorama.py on one rank: window / levels / smooth / equirect / network stream
#   clock [tag] [bench args]   effective shader clock per kernel (GRBM_GUI_ACTIVE / 8 / wall) -> profiles/<round>_<tag>_clock.json
set -o pipefail
R=${ROUND:-r06}
TASK=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out profiles

stats() {   # <kernel_stats.csv glob dir> <name filter>
  python - "$1" "$2" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if sys.argv[2] in r["Name"]:
        print(f'{float(r["AverageNs"])/1e3:8.1f} us  x{r["Calls"]:>4}  {r["Name"][:80]}')
PY
}

check() {
  export I2PC_PARITY_LOG=gpurun_out/parity.jsonl
  rm -f "$I2PC_PARITY_LOG"
  local K=()
  [ -n "$1" ] && K=(-k "$1")
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=5 --timeout 300 --timeout-method thread -rP "${K[@]}" \
    > gpurun_out/gputests.log 2>&1
  local rc=$?
  tail -5 gpurun_out/gputests.log
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || return $rc
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err
  local rc2=$?
  cut -c1-400 gpurun_out/bench.json
  return $(( rc > rc2 ? rc : rc2 ))
}

profile() {
  local TAG=$1; shift
  local D=gpurun_out/prof_$TAG
  rm -rf "$D"; mkdir -p "$D"
  timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$D/stats" -o run --output-format csv -- \
    python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-medium --strict-accounting "$@" > "$D/bench.json" 2> "$D/bench.err" \
    || { echo "stats run failed"; tail -5 "$D/bench.err"; return 1; }
  for grp in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace -d "$D/pmc" -o $grp --output-format csv -- \
      python bench.py --steps 1 --warmup 0 --no-graph --no-kernel-profile --no-cpu-baseline --no-medium "$@" > "$D/pmc_$grp.txt" 2>&1 \
      || { echo "pmc pass $grp failed"; tail -5 "$D/pmc_$grp.txt"; return 1; }
  done
  python tools/pmc_traffic.py "$D/pmc" "profiles/${R}_${TAG}_pmc_traffic.json" || return 1
  cp "$(find "$D/stats" -name '*kernel_stats.csv' | head -1)" "profiles/${R}_${TAG}_kernel_stats.csv" || return 1
  tail -1 "$D/bench.json" > "profiles/${R}_${TAG}_bench.json"
  cp profiles/${R}_${TAG}_* gpurun_out/
  echo profile_ok
}

sq() {
  local TAG=$1; shift
  local D=gpurun_out/sq_$TAG
  rm -rf "$D"; mkdir -p "$D"
  local P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"
  local P2="SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS"
  local i=0
  for grp in "$P1" "$P2"; do
    i=$((i + 1))
    timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace -d "$D/p$i" -o p$i --output-format csv -- \
      python bench.py --steps 1 --warmup 0 --no-graph --no-kernel-profile --no-cpu-baseline --no-medium "$@" > "$D/p$i.txt" 2>&1 \
      || { echo "pass $i failed"; tail -5 "$D/p$i.txt"; return 1; }
  done
  { for f in attention gemm_p; do python tools/pmc_summary.py "$D/p1" $f; python tools/pmc_summary.py "$D/p2" $f; done; } \
    > "gpurun_out/${R}_${TAG}_sq.txt" && echo sq_ok
}

case "$TASK" in
  check) check "$@" ;;
  profile) profile "$@" ;;
  sq) sq "$@" ;;
  full) check && profile dpt-large-bf16 && profile dpt-hybrid-fp8 --model dpt-hybrid --batch 64 ;;
  final1) check && cp gpurun_out/bench.json profiles/${R}_bench_check.json && cp gpurun_out/bench.json gpurun_out/${R}_bench_check.json \
          && profile dpt-large-bf16 && profile dpt-large-bf16-medium --density medium ;;
  final2) profile depth-anything-v2-small-bf16 --model depth-anything-v2 && profile dpt-hybrid-fp8 --model dpt-hybrid --batch 64 ;;
  bench)
    timeout -k 10 400 python -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
    rc=$?; cut -c1-400 gpurun_out/bench_default.json; exit $rc ;;
  ab-pipe)
    timeout -k 10 600 python -u tools/ab_pipeline.py "$@" > gpurun_out/ab_pipe.log 2>&1; rc=$?
    grep -v amdgpu.ids gpurun_out/ab_pipe.log; exit $rc ;;
  census)
    timeout -k 10 300 python -u tools/gemm_census.py "$@" > gpurun_out/census.txt 2>&1; rc=$?
    grep -v amdgpu.ids gpurun_out/census.txt; exit $rc ;;
  gemmdiag)   # census of the C2 network + per-tile s_memtime stamps of the transformer GEMMs (stamps lib prebuilt)
    timeout -k 10 300 python -u tools/gemm_census.py > gpurun_out/census.txt 2>&1 || { tail -5 gpurun_out/census.txt; exit 1; }
    head -30 gpurun_out/census.txt
    for shp in "18464 3072 1024" "18464 4096 1024 gelu" "18464 1024 1024" "18464 1024 4096"; do
      I2PC_GEMM_P=2 I2PC_LIB=image_to_pointcloud_amd/libi2pc_stamps.so timeout -k 10 120 python -u tools/stamps_p.py $shp \
        >> gpurun_out/stamps.txt 2>&1 || { tail -5 gpurun_out/stamps.txt; exit 1; }
    done
    cat gpurun_out/stamps.txt ;;
  gm)         # GROUP_M of the GEMM tile order (an XCD's 32 concurrent tiles = GROUP_M x 32 / GROUP_M): census per value
    for GM in 2 4 8 16; do
      I2PC_GEMM_GM=$GM timeout -k 10 300 python -u tools/gemm_census.py --top 12 > gpurun_out/census_gm$GM.txt 2>&1 \
        || { tail -5 gpurun_out/census_gm$GM.txt; exit 1; }
      echo "== GM $GM"; grep -v amdgpu.ids gpurun_out/census_gm$GM.txt | head -16
    done ;;
  ab-hyb)     # engine modes 0 (automatic) / 2 (persistent wherever it applies) on the DPT-Hybrid bf16 linears
    AB_SHAPES=hybrid AB_MODES=0,2 timeout -k 10 300 python -u tools/bench_gemm_ab.py > gpurun_out/ab.log 2>&1; rc=$?
    cat gpurun_out/ab.log; exit $rc ;;
  epi)        # epilogue cost of the tile GEMM on the O-projection / FC2 shapes
    timeout -k 10 300 python -u tools/epi_cost.py > gpurun_out/epi.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/epi.log; exit $rc ;;
  ab-gemm)
    timeout -k 10 300 python -u -m pytest tests/test_gemm_engines_gpu.py -x -q --timeout 120 --timeout-method thread \
      > gpurun_out/eng.log 2>&1 || { tail -15 gpurun_out/eng.log; exit 1; }
    tail -2 gpurun_out/eng.log
    timeout -k 10 300 python -u tools/bench_gemm_ab.py > gpurun_out/ab.log 2>&1; rc=$?; cat gpurun_out/ab.log; exit $rc ;;
  unp)
    timeout -k 10 400 python -u -m pytest tests/test_unproject_gpu.py -x -q --timeout 200 --timeout-method thread \
      > gpurun_out/unp_tests.log 2>&1 || { tail -15 gpurun_out/unp_tests.log; exit 1; }
    tail -2 gpurun_out/unp_tests.log
    for v in "ROWS=1 NT=1 RPT=8" "ROWS=1 NT=0 RPT=8" "ROWS=1 NT=1 RPT=4" "ROWS=0 NT=1 RPT=8"; do
      set -- $v
      env I2PC_UNP_$1 I2PC_UNP_$2 I2PC_UNP_$3 timeout -k 10 120 python tools/bench_unproject.py 32 high \
        > gpurun_out/v.txt 2>&1 || exit 1
      echo "$v: $(grep -h 'B=' gpurun_out/v.txt | sed 's/algorithmic.*//' | tr '\n' ' ')"
    done ;;
  trace-unp)
    D=gpurun_out/trace_unp${TAG}; rm -rf $D; mkdir -p $D
    timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $D/t -o t --output-format csv -- \
      python tools/bench_unproject.py ${1:-32} ${2:-high} "${@:3}" > $D/bench.txt 2>&1 || { tail -5 $D/bench.txt; exit 1; }
    grep 'B=' $D/bench.txt; stats $D/t unproj ;;
  sel-rows)   # k_sweep_w duration by output rows per workgroup (kernel trace only), then its SQ counters
    for R in 8 16 32 64; do
      D=gpurun_out/selrows_$R; rm -rf $D; mkdir -p $D
      I2PC_SEL_ROWS=$R timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $D/t -o t --output-format csv -- \
        python tools/bench_unproject.py 32 high > $D/bench.txt 2>&1 || { tail -5 $D/bench.txt; exit 1; }
      echo "rows $R: $(grep -h 'B=32 high:' $D/bench.txt)"; stats $D/t k_sweep_w
    done
    D=gpurun_out/pmc_sw; rm -rf $D; mkdir -p $D
    timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM --kernel-trace -d $D/p1 -o p1 --output-format csv -- python tools/bench_unproject.py 32 > $D/p1.txt 2>&1 || exit 1
    timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA --kernel-trace -d $D/p2 -o p2 --output-format csv -- python tools/bench_unproject.py 32 > $D/p2.txt 2>&1 || exit 1
    python tools/pmc_summary.py $D/p1 k_sweep_w && python tools/pmc_summary.py $D/p2 k_sweep_w ;;
  pmc-unp)
    D=gpurun_out/pmc_unp; rm -rf $D; mkdir -p $D
    timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --kernel-trace -d $D/p1 -o p1 --output-format csv -- python tools/bench_unproject.py 32 > $D/p1.txt 2>&1 || exit 1
    timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS --kernel-trace -d $D/p2 -o p2 --output-format csv -- python tools/bench_unproject.py 32 > $D/p2.txt 2>&1 || exit 1
    python tools/pmc_summary.py $D/p1 unproj:: && python tools/pmc_summary.py $D/p2 unproj:: ;;
  c4)         # C4 panorama, one rank: window selection (RCCL, graph), levels (host exchange), smooth, network stream
    : > gpurun_out/c4.jsonl
    for v in "--graph --check" "--levels --check" "--graph --smooth --check" "--graph --projection equirect --check" \
             "--graph --network --check"; do
      timeout -k 10 300 python -u tools/c4_panorama.py --steps 20 $v >> gpurun_out/c4.jsonl 2> gpurun_out/c4.err \
        || { tail -5 gpurun_out/c4.err; exit 1; }
    done
    cut -c1-330 gpurun_out/c4.jsonl ;;
  trace-c4)   # kernel durations of the one-rank C4 band call (window selection; args: extra c4_panorama flags)
    D=gpurun_out/trace_c4; rm -rf $D; mkdir -p $D
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/t -o t --output-format csv -- \
      python tools/c4_panorama.py --steps 10 "$@" > $D/run.txt 2>&1 || { tail -5 $D/run.txt; exit 1; }
    grep -o '"ms_per_image": [0-9.]*' $D/run.txt; stats $D/t unproj ;;
  parts)      # whole unprojection call by selection sub-batches (I2PC_SEL_PARTS), then the kernel trace at the default
    for P in 1 2 3 4; do
      I2PC_SEL_PARTS=$P timeout -k 10 120 python tools/bench_unproject.py 32 high > gpurun_out/v.txt 2>&1 || exit 1
      echo "parts $P: $(grep -h 'B=' gpurun_out/v.txt | sed 's/algorithmic.*//' | tr '\n' ' ')"
    done ;;
  pmc-sweep)  # SQ counters of k_sweep_w: the C2 batch call and the one-rank C4 band call
    D=gpurun_out/pmc_sweep; rm -rf $D; mkdir -p $D
    P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM"
    P2="SQ_WAVES SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA"
    i=0
    for P in "$P1" "$P2"; do
      i=$((i + 1))
      timeout -k 10 120 rocprofv3 --pmc $P --kernel-trace -d $D/u$i -o u --output-format csv -- python tools/bench_unproject.py 32 > $D/u$i.txt 2>&1 || exit 1
      timeout -k 10 120 rocprofv3 --pmc $P --kernel-trace -d $D/c$i -o c --output-format csv -- python tools/c4_panorama.py --steps 2 --warmup 1 > $D/c$i.txt 2>&1 || exit 1
    done
    for i in 1 2; do echo "== C2 pass $i"; python tools/pmc_summary.py $D/u$i k_sweep_w; echo "== C4 pass $i"; python tools/pmc_summary.py $D/c$i k_sweep_w; done ;;
  clock)      # effective shader clock per kernel (GRBM_GUI_ACTIVE / 8 / wall; DVFS give-back) of the bench network
    TAG=${1:-dpt-large-bf16}; shift || true
    D=gpurun_out/clock_$TAG; rm -rf $D; mkdir -p $D
    timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace -d $D/p -o p --output-format csv -- \
      python bench.py --steps 3 --warmup 0 --no-graph --no-kernel-profile --no-cpu-baseline "$@" > $D/run.txt 2>&1 \
      || { tail -5 $D/run.txt; exit 1; }
    python tools/pmc_clock.py $D/p "profiles/${R}_${TAG}_clock.json" && cp "profiles/${R}_${TAG}_clock.json" gpurun_out/ ;;
  *) echo "unknown task '$TASK' (see the header of tools/gpu.sh)"; exit 2 ;;
esac
