#!/bin/bash
# dev: the full-size configs (C3, C4, C5) with different batch sizes (RS_MAX_BATCH_ITEMS: camera
# samples in flight per wavefront batch) and lane counts; tools/time_scene.py best of 3 frames.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-batch}; mkdir -p $OUT; cd $R
run() { local tag=$1; shift; echo "== $tag" >> $OUT/batch.txt; env "$@" timeout -k 10 300 python tools/time_scene.py default ${SC} >> $OUT/batch.txt 2>&1 || { echo "$tag failed"; tail -5 $OUT/batch.txt; exit 1; }; }
SC="mesh 484 50 1920x1080"
run c5_b32M RS_MAX_BATCH_ITEMS=33554432
run c5_b128M RS_MAX_BATCH_ITEMS=134217728
run c5_b128M_l4 RS_MAX_BATCH_ITEMS=134217728 RS_LANES=4
SC="quadric 1024 50 1024x1024"
run c4_b32M RS_MAX_BATCH_ITEMS=33554432
run c4_b128M RS_MAX_BATCH_ITEMS=134217728
cat $OUT/batch.txt | grep -v "^W2026\|amdgpu.ids"
echo done
