#!/bin/bash
# One GPU-box session of per-scene profiles: rocprofv3 kernel traces of the C4 and C5 configs' scenes
# (tools/time_scene.py at reduced spp) and the instruction-mix / lane-utilisation PMC passes
# (tools/pmc_mix.sh) on the bench frame, C4's and C5's scenes. Outputs under gpurun_out/<tag>/.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-scenes}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/tr_c4 -o tr -- python3 $R/tools/time_scene.py default quadric 16 50 1024x1024 > $OUT/tr_c4.log 2>&1 || { echo "c4 trace failed"; tail -5 $OUT/tr_c4.log; exit 1; }
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/tr_c5 -o tr -- python3 $R/tools/time_scene.py default mesh 16 50 1920x1080 > $OUT/tr_c5.log 2>&1 || { echo "c5 trace failed"; tail -5 $OUT/tr_c5.log; exit 1; }
cd $R
for sc in "rtow 64 8" "quadric_sdl 16 50" "mesh_scene 16 50"; do
  set -- $sc
  bash tools/pmc_mix.sh $OUT/mix_$1 - $1 $2 $3 > $OUT/mix_$1.log 2>&1 || { echo "pmc $1 failed"; tail -5 $OUT/mix_$1.log; exit 1; }
  python tools/pmc_mix.py $OUT/mix_$1 $OUT/mix_$1.json > $OUT/mix_$1.txt 2>&1
done
cat $OUT/mix_*.txt
echo done
