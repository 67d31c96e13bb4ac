#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r3f}; mkdir -p $OUT; cd $R
L=$R/raysnail_amd/lib
timeout -k 10 900 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > $OUT/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
timeout -k 10 600 python tools/variant_share.py $L/libraysnail_hip.so $L/var_ext5.so $L/var_gen4.so $L/var_ext5gen4.so > $OUT/variants.txt 2>&1 || { echo "variants failed"; cat $OUT/variants.txt; exit 1; }
timeout -k 10 600 python tools/bench_configs.py --only C2,C4 --cpu-seconds 2 > $OUT/configs.jsonl 2> $OUT/configs.err || { echo "configs failed"; tail -5 $OUT/configs.err; exit 1; }
echo done
