set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python tools/bench_torch_ref.py > gpurun_out/calib.log 2>&1 || { echo calib_failed; exit 1; }
timeout -k 10 300 python tools/bench_gemm.py > gpurun_out/gemm_ours.log 2>&1 || { echo gemm_failed; exit 1; }
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/bench2.json 2> gpurun_out/bench2.err || { echo bench_failed; exit 1; }
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof2 -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof2.log 2>&1 || { echo prof_failed; exit 1; }
echo all_ok
