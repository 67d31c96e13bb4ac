#!/bin/bash
# dev: A/B of library builds on several scenes (tools/variant_bench.py) and of wavefront lane counts
# on the bench frame and its N=8 row share (tools/variant_share.py).
# usage: tools/gpu_variants.sh <tag> "<scenes>" <lib.so[:ENV=v]>... ; outputs under gpurun_out/<tag>/
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1; SCN=$2; shift 2; mkdir -p $OUT; cd $R; export TMPDIR=/tmp
for sc in $SCN; do
  if [ "$sc" = share ]; then
    timeout -k 10 400 python tools/variant_share.py "$@" > $OUT/share.txt 2>&1 || { echo "share failed"; cat $OUT/share.txt; exit 1; }
    cat $OUT/share.txt
  else
    timeout -k 10 400 python tools/variant_bench.py --scene=$sc "$@" > $OUT/$sc.txt 2>&1 || { echo "$sc failed"; cat $OUT/$sc.txt; exit 1; }
    cat $OUT/$sc.txt
  fi
done
echo done
