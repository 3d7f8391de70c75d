# skinny GEMM without the row guard: its tests, in-process A/B against the tile kernel, census
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_engines_gpu.py -x -q -k skinny --timeout 200 --timeout-method thread > gpurun_out/t29.log 2>&1 || { tail -30 gpurun_out/t29.log; exit 1; }
tail -1 gpurun_out/t29.log
bash tools/gpu.sh ab-pipe --rounds 4 --variant base: --variant skinny:gemm_skinny=1 || exit 1
I2PC_GEMM_SKINNY=1 bash tools/gpu.sh census --top 60 > gpurun_out/census29.txt 2>&1 || exit 1
grep "skinny\|m32 \|network launches" gpurun_out/census29.txt
