#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r3h}; mkdir -p $OUT; cd $R
L=$R/raysnail_amd/lib
timeout -k 10 300 python tools/trav_stats.py $L/var_stats.so rtow,mesh,example,quadric > $OUT/trav_stats.txt 2>&1 || { echo "trav stats failed"; cat $OUT/trav_stats.txt; exit 1; }
timeout -k 10 600 python tools/variant_bench.py --scene=c5 $L/libraysnail_hip.so $L/var_ltri0.so > $OUT/variants_c5.txt 2>&1 || { echo "c5 variants failed"; cat $OUT/variants_c5.txt; exit 1; }
timeout -k 10 900 python tools/bench_configs.py --only C2,C4,C5 --cpu-seconds 2 > $OUT/configs.jsonl 2> $OUT/configs.err || { echo "configs failed"; tail -5 $OUT/configs.err; exit 1; }
echo done
