#!/bin/bash
# dev: rocprofv3 kernel traces of the bench frame (tools/render_once.py, 5 frames) and of the N=8 row
# share (tools/share_frames.py, 10 frames) for dev-library configurations; per-bounce tables printed.
# usage: tools/trace_ab.sh <outdir> "ENV=v ..." ["ENV=v ..."]
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$1; shift; case $OUT in /*) ;; *) OUT=$R/$OUT;; esac
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
k=0
for cfg in "$@"; do
  k=$((k+1))
  env RS_HIP_LIB=$R/raysnail_amd/lib/libraysnail_hip_dev.so $cfg timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/full$k -o full -- python3 $R/tools/render_once.py 0 5 > $OUT/full$k.log 2>&1 || { echo "$cfg full trace FAILED"; exit 1; }
  env RS_HIP_LIB=$R/raysnail_amd/lib/libraysnail_hip_dev.so $cfg timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/share$k -o share -- python3 $R/tools/share_frames.py 8 10 > $OUT/share$k.log 2>&1 || { echo "$cfg share trace FAILED"; exit 1; }
  echo "== $cfg" >> $OUT/cfgs.txt
  echo "$k: $cfg  $(tail -1 $OUT/full$k.log) | $(tail -1 $OUT/share$k.log)"
done
