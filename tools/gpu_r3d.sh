#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r3d}; mkdir -p $OUT; cd $R
L=$R/raysnail_amd/lib/libraysnail_hip.so
timeout -k 10 900 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > $OUT/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
timeout -k 10 600 python tools/variant_share.py $L:RS_TAIL_PATHS=0 $L:RS_TAIL_PATHS=65536 $L:RS_TAIL_PATHS=131072 $L:RS_TAIL_PATHS=262144 $L:RS_TAIL_PATHS=524288 $L:RS_TAIL_PATHS=1048576 > $OUT/variants.txt 2>&1 || { echo "variants failed"; cat $OUT/variants.txt; exit 1; }
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/share -o share -- python3 $R/tools/share_frames.py 8 10 > $OUT/share_frames.log 2> $OUT/share.err || { echo "share trace failed"; exit 1; }
echo done
