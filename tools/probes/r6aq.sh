set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for r in 1 2 3; do
  echo "== session $r"
  timeout -k 10 240 python -u tools/probes/det_ops2.py 4 8 2>&1 | grep "^proc" || exit 1
done
