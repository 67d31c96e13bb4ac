#!/bin/bash
# One-lane bench frames (tools/render_once.py, RS_LANES=1): PMC instruction-mix passes and a kernel
# trace of the same command, then the VALU-issue roofline per kernel (tools/valu_roofline.py).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-valu}; mkdir -p $OUT
export RS_LANES=1
bash $R/tools/pmc_mix.sh $OUT/mix - ${2:-rtow} ${3:-64} ${4:-8} > $OUT/mix.log 2>&1 || { echo "pmc failed"; tail -5 $OUT/mix.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr -o tr -- python3 $R/tools/render_once.py 0 2 ${2:-rtow} ${3:-64} ${4:-8} > $OUT/tr.log 2>&1 || { echo "trace failed"; exit 1; }
cd $R
python tools/valu_roofline.py $OUT/mix $(ls $OUT/tr/*kernel_trace.csv) $OUT/valu_roofline.json
echo done
