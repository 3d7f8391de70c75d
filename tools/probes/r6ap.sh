set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
run() { echo "== $*"; env "$@" timeout -k 10 200 python -u tools/det_rep.py 4 10 0 2>&1 | grep "^proc" || exit 1; }
for r in 1 2; do
  run DET_KNOBS=
  run DET_KNOBS=gemm_resq=1,gemm_simple_epi=0,attn_rb=0
  run DET_KNOBS=gemm_stagger=0
done
