#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r3k}; mkdir -p $OUT; cd $R; export TMPDIR=/tmp
L=$R/raysnail_amd/lib
timeout -k 10 600 python tools/variant_bench.py --scene=c5 $L/var_lq0.so $L/libraysnail_hip.so $L/var_thr32.so $L/var_thr56.so $L/var_thr64.so > $OUT/leafq_c5.txt 2>&1 || { echo "c5 variants failed"; cat $OUT/leafq_c5.txt; exit 1; }
cat $OUT/leafq_c5.txt
timeout -k 10 300 python tools/trav_stats.py $L/var_stats0.so mesh > $OUT/trav_stats0.txt 2>&1 || { echo "trav stats failed"; cat $OUT/trav_stats0.txt; exit 1; }
timeout -k 10 300 python tools/trav_stats.py $L/var_stats.so mesh > $OUT/trav_stats.txt 2>&1 || { echo "trav stats failed"; cat $OUT/trav_stats.txt; exit 1; }
cat $OUT/trav_stats0.txt $OUT/trav_stats.txt
bash tools/pmc_mix.sh $OUT/mix_c5 - mesh_scene 16 50 > $OUT/mix_c5.log 2>&1 || { echo "pmc failed"; cat $OUT/mix_c5.log; exit 1; }
python tools/pmc_mix.py $OUT/mix_c5 $OUT/mix_c5.json > /dev/null 2>&1
echo done
