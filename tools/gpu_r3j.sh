#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r3j}; mkdir -p $OUT; cd $R; export TMPDIR=/tmp
L=$R/raysnail_amd/lib/libraysnail_hip.so
timeout -k 10 600 python tools/variant_bench.py --scene=c5 $L $L:RS_PHASES=24 $L:RS_PHASES=16 $L:RS_PHASES=32 $L:RS_PHASES=16/16 $L:RS_PHASES=24/16 $L:RS_PHASES=12/12/12 $L:RS_PHASES=1 > $OUT/phases_c5.txt 2>&1 || { echo "c5 variants failed"; cat $OUT/phases_c5.txt; exit 1; }
cat $OUT/phases_c5.txt
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/c5 -o c5 --output-format csv -- python tools/bounce_trace.py c5 1 > $OUT/c5.log 2>&1 || { echo "c5 trace failed"; tail -20 $OUT/c5.log; exit 1; }
F=$(find $OUT/c5 -name '*kernel_trace.csv' | head -1)
python tools/bounce_trace.py --report $F 50 > $OUT/c5_bounces.txt 2>&1
echo done
