#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r3e}; mkdir -p $OUT; cd $R
timeout -k 10 900 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > $OUT/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
bash tools/pmc_mix.sh $OUT/mix list > $OUT/mix.log 2>&1 || { echo "pmc mix failed"; cat $OUT/mix.log; exit 1; }
bash tools/pmc_mix.sh $OUT/mix_c4 - quadric_sdl 16 > $OUT/mix_c4.log 2>&1 || { echo "pmc mix c4 failed"; cat $OUT/mix_c4.log; exit 1; }
bash tools/pmc_mix.sh $OUT/mix_c5 - mesh_scene 16 > $OUT/mix_c5.log 2>&1 || { echo "pmc mix c5 failed"; cat $OUT/mix_c5.log; exit 1; }
timeout -k 10 900 python tools/bench_configs.py --only C2,C4,C5,X1,X2 --cpu-seconds 3 > $OUT/configs.jsonl 2> $OUT/configs.err || { echo "configs failed"; tail -5 $OUT/configs.err; exit 1; }
L=$R/raysnail_amd/lib
timeout -k 10 600 python tools/variant_bench.py --scene=c5 $L/libraysnail_hip.so $L/var_notri.so > $OUT/variants_c5.txt 2>&1 || { echo "c5 variants failed"; cat $OUT/variants_c5.txt; exit 1; }
echo done
