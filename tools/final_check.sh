R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/final3; mkdir -p $OUT
cd $R && timeout -k 10 600 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > $OUT/pytest.log 2>&1 || { tail -20 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -10 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
timeout -k 10 300 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -10 $OUT/bench.err; exit 1; }
tail -1 $OUT/bench.json | cut -c1-300
timeout -k 10 900 python3 tools/bench_configs.py > $OUT/configs.jsonl 2> $OUT/configs.err || { tail -5 $OUT/configs.err; exit 1; }
python3 -c "
import json
for l in open('$OUT/configs.jsonl'):
    d=json.loads(l); g=d['gpu']; print(d['config'], g['Msamples_per_s'], round(g['Msamples_per_s']*g['segments_per_sample']/1000,3), g['ms_per_frame'], d['speedup'], d['sampled_rows_bit_identical'])"
