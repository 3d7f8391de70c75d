cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for cfg in "32 medium" "32 high 512 512 384 384"; do
  for rpt in 8 4 2 1; do
    D=gpurun_out/t18; rm -rf $D; mkdir -p $D
    I2PC_UNP_RPT=$rpt timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $D -o t --output-format csv -- python tools/bench_unproject.py $cfg > $D/b.txt 2>&1 || { tail -3 $D/b.txt; exit 1; }
    k=$(python -c "
import csv,glob
f=glob.glob('$D/**/*kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'k_unproject_rows' in r['Name']: print(round(float(r['AverageNs'])/1e3,1))")
    echo "cfg [$cfg] rpt $rpt: k_unproject_rows $k us; $(grep -h 'B=' $D/b.txt | head -1 | sed 's/algorithmic.*//')"
  done
done
