#!/bin/bash
# dev: same-box kernel traces of the bench frame, baseline (the git worktree base/, see tools/ab_base.sh) then this tree's dev library
# per configuration; per-bounce table via tools/trace_cmp.py
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$1; shift; case $OUT in /*) ;; *) OUT=$R/$OUT;; esac
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
(cd $R/base && RS_LANES=1 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/base -o t -- python3 $R/base/tools/render_once.py 0 5 > $OUT/base.log 2>&1) || { echo "base trace FAILED"; exit 1; }
k=0
for cfg in "$@"; do
  k=$((k+1))
  env RS_HIP_LIB=$R/raysnail_amd/lib/libraysnail_hip_dev.so $cfg timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/v$k -o t -- python3 $R/tools/render_once.py 0 5 > $OUT/v$k.log 2>&1 || { echo "$cfg trace FAILED"; exit 1; }
done
echo done
