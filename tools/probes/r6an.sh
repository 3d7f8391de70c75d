set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
P=$PWD/image_to_pointcloud_amd/libi2pc_prev.so
C=$PWD/image_to_pointcloud_amd/libi2pc.so
for r in 1 2 3; do
  for lib in $C $P; do
    echo "== $r $(basename $lib)"
    I2PC_LIB=$lib timeout -k 10 200 python -u tools/det_rep.py 2 10 0 2>&1 | grep "^proc" || exit 1
  done
done
