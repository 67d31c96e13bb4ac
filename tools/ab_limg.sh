#!/bin/bash
# dev: the nest modes' LDS scene image (DScene::limg) against the global tables (RS_NO_LIMG, dev
# library): frame times and kernel stats of C4's and C2's scenes
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/${1:-limg}; mkdir -p $OUT
DEV=$R/raysnail_amd/lib/libraysnail_hip_dev.so
cd /tmp && export TMPDIR=/tmp
for sc in "quadric 16 50 1024x1024" "example 64 50 800x500"; do
  set -- $sc
  for mode in lds glob; do
    if [ $mode = glob ]; then export RS_NO_LIMG=1; else unset RS_NO_LIMG; fi
    timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/tr_$1_$mode -o tr -- python3 $R/tools/time_scene.py $DEV $1 $2 $3 $4 > $OUT/$1_$mode.log 2>&1 || { echo "$1 $mode FAILED"; tail -5 $OUT/$1_$mode.log; exit 1; }
    echo "== $1 $mode $(tail -1 $OUT/$1_$mode.log)" >> $OUT/ab.txt
    python3 -c "
import csv,glob
f=glob.glob('$OUT/tr_$1_$mode/**/*kernel_stats.csv',recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:4]: print('   %-60s n=%5s avg %9.1f us  %5.1f%%' % (r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e3, float(r['Percentage'])))
" >> $OUT/ab.txt
  done
done
unset RS_NO_LIMG
cat $OUT/ab.txt
