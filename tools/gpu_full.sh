# Full GPU pass: every -m gpu test, smoke(), the default bench line, and a rocprofv3 kernel-stats run of the bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -v -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/t_all.log 2>&1 || { echo tests_failed; tail -40 gpurun_out/t_all.log; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke_failed; tail -20 gpurun_out/smoke.log; exit 1; }
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo bench_failed; tail -20 gpurun_out/bench.err; exit 1; }
timeout -k 10 600 python bench.py --density medium --no-cpu-baseline > gpurun_out/bench_medium.json 2> gpurun_out/bench_medium.err || { echo bench_medium_failed; tail -20 gpurun_out/bench_medium.err; exit 1; }
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1 || { echo prof_failed; exit 1; }
echo all_ok
