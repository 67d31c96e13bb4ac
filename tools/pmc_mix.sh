#!/bin/bash
# Instruction-mix / wait / lane-utilisation counter passes on the bench frame (tools/render_once.py),
# one rocprofv3 --pmc run per pass (each within the per-block limits: <= 8 SQ counters).
# usage: tools/pmc_mix.sh <outdir> [list|-] [scene] [spp] [depth] -> <outdir>/pN/**/counter_collection.csv
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$1; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
if [ "${2:-}" = "list" ]; then timeout -s KILL 90 rocprofv3 -L > $OUT/counters.txt 2>&1 || echo "list failed (ignored)"; fi
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_FMA_F64" \
           "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT" \
           "SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT" \
           "TCC_HIT_sum TCC_MISS_sum" ; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $OUT/p$i -o pmc -- python3 $R/tools/render_once.py 0 2 ${3:-rtow} ${4:-64} ${5:-8} > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
echo done
