#!/bin/bash
# dev: one scene timed with the in-tree build and with the builds of earlier commits (git worktrees
# wt_<commit>/ built in place), each through its own tools/variant_bench.py; env variants of the
# current build after them. usage: tools/gpu_bisect.sh <tag> <scene> [wt dirs...]
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1; SC=$2; shift 2; mkdir -p $OUT; cd $R; export TMPDIR=/tmp
L=$R/raysnail_amd/lib
for w in "$@"; do
  timeout -k 10 300 python $w/tools/variant_bench.py --scene=$SC > $OUT/$w.txt 2>&1 || { echo "$w failed"; cat $OUT/$w.txt; exit 1; }
  cat $OUT/$w.txt
done
timeout -k 10 300 python tools/variant_bench.py --scene=$SC $L/libraysnail_hip.so $L/libraysnail_hip.so:RS_LANES=1 > $OUT/cur.txt 2>&1 || { echo "cur failed"; cat $OUT/cur.txt; exit 1; }
cat $OUT/cur.txt
echo done
