#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r3g}; mkdir -p $OUT; cd $R
L=$R/raysnail_amd/lib
timeout -k 10 900 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > $OUT/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
timeout -k 10 600 python tools/variant_share.py $L/libraysnail_hip.so $L/var_nolw.so $L/libraysnail_hip.so $L/var_nolw.so > $OUT/variants.txt 2>&1 || { echo "variants failed"; cat $OUT/variants.txt; exit 1; }
timeout -k 10 600 python tools/variant_bench.py --scene=c4 $L/libraysnail_hip.so $L/var_nolw.so > $OUT/variants_c4.txt 2>&1 || { echo "c4 variants failed"; cat $OUT/variants_c4.txt; exit 1; }
timeout -k 10 600 python tools/variant_bench.py --scene=example $L/libraysnail_hip.so $L/var_nolw.so > $OUT/variants_c2.txt 2>&1 || { echo "c2 variants failed"; cat $OUT/variants_c2.txt; exit 1; }
echo done
