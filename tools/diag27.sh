# skinny GEMM (M <= 64 rows: the CLS readout): engine tests, network parity, in-process A/B, census
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gemm_engines_gpu.py tests/test_dpt_gpu.py tests/test_abi.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t27.log 2>&1 || { tail -30 gpurun_out/t27.log; exit 1; }
tail -1 gpurun_out/t27.log
bash tools/gpu.sh ab-pipe --rounds 4 --variant base: --variant noskinny:gemm_skinny=0 || exit 1
bash tools/gpu.sh census --top 60 > gpurun_out/census27.txt 2>&1 || exit 1
grep "skinny\|m32 \|network launches" gpurun_out/census27.txt
