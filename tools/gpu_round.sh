#!/bin/bash
# One GPU-box session: tests -> rocprofv3 kernel trace -> PMC passes (FETCH_SIZE, WRITE_SIZE) -> PMC
# summary (profiles/pmc_summary.json) -> bench (with CPU baseline, reading that summary) -> config sweep. Every GPU step has its own time limit; the script stops at
# the first failure. Outputs under gpurun_out/<tag>/ (copy what is judged into profiles/).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-round}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
step() { local t=$1; shift; echo "== $* (limit ${t}s)" >> $OUT/steps.log; timeout -k 10 $t "$@"; local rc=$?; echo "   rc=$rc" >> $OUT/steps.log; return $rc; }
step 600 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > $OUT/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
step 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 $R/bench.py --steps 5 --warmup 2 --cpu-baseline 0 --row-share 0 > $OUT/bench_under_rocprof.json 2> $OUT/prof_bench.err || { echo "rocprof trace failed"; exit 1; }
step 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o pmc -- python3 $R/bench.py --steps 3 --warmup 1 --cpu-baseline 0 --row-share 0 > /dev/null 2> $OUT/pmc_fetch.err || { echo "pmc fetch failed"; exit 1; }
step 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o pmc -- python3 $R/bench.py --steps 3 --warmup 1 --cpu-baseline 0 --row-share 0 > /dev/null 2> $OUT/pmc_write.err || { echo "pmc write failed"; exit 1; }
cd $R
# the bench line's roofline.traffic is read from profiles/pmc_summary.json: refresh it from this build's passes first
FC=$(find $OUT/pmc_fetch -name '*counter_collection.csv' | head -1); WC=$(find $OUT/pmc_write -name '*counter_collection.csv' | head -1)
python tools/collect_pmc.py "$FC" "$WC" $R/profiles/pmc_summary.json $TAG && cp $R/profiles/pmc_summary.json $OUT/pmc_summary_wavefront.json || { echo "pmc summary failed"; exit 1; }
step 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
cd $R
step 900 python tools/bench_configs.py > $OUT/configs.jsonl 2> $OUT/configs.err || { echo "config sweep failed"; tail -5 $OUT/configs.err; exit 1; }
echo done
