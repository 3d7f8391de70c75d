set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for r in 1 2 3; do
  echo "== session $r"
  timeout -k 10 240 python -u tools/probes/det_ops2.py 4 8 2>&1 | grep "^proc" || exit 1
done
for r in 1 2; do
  echo "== det_rep 4 $r"
  timeout -k 10 200 python -u tools/det_rep.py 4 10 0 2>&1 | grep "^proc" || exit 1
done
timeout -k 10 400 python -u -m pytest -q --timeout 240 --timeout-method thread -m gpu tests/test_ln_fold_gpu.py \
  tests/test_gemm_engines_gpu.py tests/test_depth_anything_gpu.py tests/test_determinism_gpu.py > gpurun_out/r6ar.log 2>&1
rc=$?; tail -3 gpurun_out/r6ar.log; exit $rc
