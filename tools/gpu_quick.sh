#!/bin/bash
# Quick GPU-box session: -m gpu tests -> bench (with the N=8 row share) -> kernel traces of the bench
# frame and of the rows 0::8 share. Outputs under gpurun_out/<tag>/. Stops at the first failure.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-quick}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
step() { local t=$1; shift; echo "== $* (limit ${t}s)" >> $OUT/steps.log; timeout -k 10 $t "$@"; local rc=$?; echo "   rc=$rc" >> $OUT/steps.log; return $rc; }
if [ "${SKIP_TESTS:-0}" != 1 ]; then
step 900 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > $OUT/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
fi
step 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
cd /tmp && export TMPDIR=/tmp
step 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 $R/tools/render_once.py 0 5 > $OUT/trace_frames.log 2> $OUT/trace.err || { echo "rocprof trace failed"; exit 1; }
step 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/share -o share -- python3 $R/tools/share_frames.py 8 10 > $OUT/share_frames.log 2> $OUT/share.err || { echo "rocprof share trace failed"; exit 1; }
echo done
