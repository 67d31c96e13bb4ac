#!/bin/bash
# dev: same-box A/B against the baseline build (a git worktree at base/: `git worktree add --detach base <rev> && make -C base/raysnail_amd/csrc`): its bench
# line, then bench_ab.sh configurations of this tree's dev library, repeated `reps` times interleaved.
# usage: tools/ab_base.sh <outdir> <reps> "ENV=v ..." ["ENV=v ..."]
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$1; shift; case $OUT in /*) ;; *) OUT=$R/$OUT;; esac
REPS=$1; shift
mkdir -p $OUT
for rep in $(seq $REPS); do
  (cd $R/base && timeout -k 10 240 python3 bench.py --cpu-baseline 0 --steps 20 --warmup 5 > $OUT/base.json 2> $OUT/base.err) || { echo "base FAILED"; tail -5 $OUT/base.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$OUT/base.json').read().strip().splitlines()[-1]); r=d.get('row_share',{})
print('baseline'.ljust(40), 'full %.3f ms  share %.4f ms  eff %.3f  value %.1f' % (d['ms_per_step'], r.get('ms_per_share',0), r.get('predicted_efficiency',0), d['value']))" | tee -a $OUT/ab.txt
  bash $R/tools/bench_ab.sh $OUT "$@" || exit 1
done
