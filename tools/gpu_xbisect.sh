#!/bin/bash
# dev: X1 / X2 (rich generic mode) timed with the in-tree build and with earlier commits' builds
# (git worktrees wt_<commit>/, built in place). usage: tools/gpu_xbisect.sh <tag> <tree>...
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1; shift; mkdir -p $OUT; cd $R
for w in "$@"; do
  timeout -k 10 240 python tools/x_time.py $w >> $OUT/x.txt 2>$OUT/x_$w.err || { echo "$w failed"; tail -5 $OUT/x_$w.err; exit 1; }
done
cat $OUT/x.txt
