#!/bin/bash
# dev: C4 / C2 against the round-2 tree (a git worktree of 1c6b7d4 at wt_r2/, built in place) and
# the merged-shading variants; kernel traces of the C4-shaped frame for both trees.
# usage: tools/gpu_cmp_r2.sh <tag>   (outputs under gpurun_out/<tag>/)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-cmp}; mkdir -p $OUT; cd $R; export TMPDIR=/tmp
L=$R/raysnail_amd/lib
for sc in c4 example; do
  timeout -k 10 300 python wt_r2/tools/variant_bench.py --scene=$sc > $OUT/r2_$sc.txt 2>&1 || { echo "r2 $sc failed"; cat $OUT/r2_$sc.txt; exit 1; }
  timeout -k 10 300 python tools/variant_bench.py --scene=$sc $L/libraysnail_hip.so $L/var_m0.so $L/var_m2.so > $OUT/cur_$sc.txt 2>&1 || { echo "cur $sc failed"; cat $OUT/cur_$sc.txt; exit 1; }
done
cat $OUT/r2_*.txt $OUT/cur_*.txt
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/tr_cur -o tr -- python3 $R/tools/time_scene.py default quadric 64 50 512x512 > $OUT/tr_cur.log 2>&1 || { echo "trace cur failed"; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/tr_r2 -o tr -- python3 $R/wt_r2/tools/time_scene.py default quadric 64 50 512x512 > $OUT/tr_r2.log 2>&1 || { echo "trace r2 failed"; exit 1; }
echo done
