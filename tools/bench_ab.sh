#!/bin/bash
# dev: bench.py A/B over tuning overrides of the dev library (libraysnail_hip_dev.so reads RS_* knobs:
# RS_FRAMES, RS_INJECT_DIV, RS_POOL_PATHS, RS_LANES, RS_MAX_BATCH_ITEMS). One line per config.
# usage: tools/bench_ab.sh <outdir> "ENV=v ENV=v" ["ENV=v" ...]      (each arg is one configuration)
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$1; shift; case $OUT in /*) ;; *) OUT=$R/$OUT;; esac
mkdir -p $OUT
for cfg in "$@"; do
  env RS_HIP_LIB=$R/raysnail_amd/lib/libraysnail_hip_dev.so $cfg timeout -k 10 240 python3 $R/bench.py --cpu-baseline 0 --steps 20 --warmup 5 > $OUT/b.json 2> $OUT/b.err || { echo "$cfg: FAILED"; tail -5 $OUT/b.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); r=d.get('row_share',{})
print('$cfg'.ljust(40), 'full %.3f ms  share %.4f ms  eff %.3f  value %.1f  extend %.4f ms/launch' % (d['ms_per_step'], r.get('ms_per_share',0), r.get('predicted_efficiency',0), d['value'], d['roofline']['avg_launch_ms']))
" | tee -a $OUT/ab.txt
done
