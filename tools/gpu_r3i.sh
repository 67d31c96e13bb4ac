#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r3i}; mkdir -p $OUT; cd $R; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/c5 -o c5 --output-format csv -- python tools/bounce_trace.py c5 1 > $OUT/c5.log 2>&1 || { echo "c5 trace failed"; tail -20 $OUT/c5.log; exit 1; }
F=$(find $OUT/c5 -name '*kernel_trace.csv' | head -1)
python tools/bounce_trace.py --report $F 50 > $OUT/c5_bounces.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/c4 -o c4 --output-format csv -- python tools/bounce_trace.py c4 1 > $OUT/c4.log 2>&1 || { echo "c4 trace failed"; tail -20 $OUT/c4.log; exit 1; }
F=$(find $OUT/c4 -name '*kernel_trace.csv' | head -1)
python tools/bounce_trace.py --report $F 50 > $OUT/c4_bounces.txt 2>&1
echo done
