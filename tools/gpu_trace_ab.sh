#!/bin/bash
# dev: rocprofv3 kernel traces of the bench frame (tools/render_once.py, one wavefront lane) for
# several library builds, and the per-kernel totals of each. usage: tools/gpu_trace_ab.sh <tag> <lib.so>...
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1; shift; mkdir -p $OUT; cd /tmp; export TMPDIR=/tmp
for lib in "$@"; do
  n=$(basename $lib .so)
  RS_HIP_LIB=$R/$lib RS_LANES=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$n -o tr -- python3 $R/tools/render_once.py 0 6 ${SCENE:-rtow} ${SPP:-64} ${DEPTH:-8} > $OUT/$n.log 2>&1 || { echo "$n trace failed"; tail -5 $OUT/$n.log; exit 1; }
  echo "== $n"; python3 $R/tools/bounce_trace.py --report $(ls $OUT/$n/*kernel_trace.csv) ${DEPTH:-8} | head -12
done
echo done
