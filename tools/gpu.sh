#!/bin/bash
# GPU-box sessions (one parameterised script; outputs under gpurun_out/<tag>/, copy what is judged into
# profiles/). Every GPU step has its own time limit and the session stops at the first failure.
# usage: bash tools/gpu.sh <tag> <step> [<step> ...]
#   tests    pytest -m gpu (every GPU test)
#   bench    python bench.py (the driver's line: CPU baseline, row share)
#   trace    rocprofv3 kernel traces: bench frames (tools/render_once.py) and N=8 row-share frames
#            (tools/share_frames.py) -> kernel_stats / kernel_trace csv
#   pmc      FETCH_SIZE / WRITE_SIZE passes over bench frames + profiles/pmc_summary.json (tools/collect_pmc.py)
#   calib    FETCH_SIZE / WRITE_SIZE / TCC_EA0_RDREQ passes over tools/micro/pmc_calib (known byte counts)
#   l1       L1 / L2 hit counters over bench frames (TCP / TCC)
#   mix      instruction-mix / lane-utilisation PMC passes (tools/pmc_mix.sh) + VALU roofline (tools/valu_roofline.py)
#            on the bench frame, C4's and C5's scenes
#   scenes   kernel traces of the C4 / C5 scenes (tools/time_scene.py)
#   configs  tools/bench_configs.py (C2-C5, X1, X2 vs the CPU oracle on row subsets)
#   ab       bench.py of this tree against the baseline worktree base/, 3 rounds interleaved (tools/ab_report.py)
#   variants bench.py of base/, the product and every raysnail_amd/lib/var_*.so (tools/build_variant.sh), 2 rounds
#   travstats per-category traversal counters (raysnail_amd/lib/trav_stats.so, a -DRS_TRAV_STATS build)
#   abtrace  kernel traces of the bench frames, base/ then this tree (tools/trace_cmp.py)
#   iters    per-iteration queue counts + extend / shading launches of the bench frame (dev library; tools/iter_table.py)
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; shift
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
step() { local t=$1; shift; echo "== $* (limit ${t}s)" >> $OUT/steps.log; timeout -k 10 $t "$@"; local rc=$?; echo "   rc=$rc" >> $OUT/steps.log; return $rc; }
for s in "$@"; do
  case $s in
  tests)
    (cd $R && step 900 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > $OUT/pytest_gpu.log 2>&1) || { echo "gpu tests failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
    tail -1 $OUT/pytest_gpu.log ;;
  bench)
    (cd $R && step 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err) || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
    tail -1 $OUT/bench.json ;;
  trace)
    (cd /tmp && step 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 $R/tools/render_once.py 0 5 > $OUT/trace_frames.log 2>&1) || { echo "trace failed"; exit 1; }
    (cd /tmp && step 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/share -o share -- python3 $R/tools/share_frames.py 8 10 > $OUT/share_frames.log 2>&1) || { echo "share trace failed"; exit 1; } ;;
  pmc)
    (cd /tmp && step 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o pmc -- python3 $R/bench.py --steps 3 --warmup 1 --cpu-baseline 0 --row-share 0 > /dev/null 2> $OUT/pmc_fetch.err) || { echo "pmc fetch failed"; exit 1; }
    (cd /tmp && step 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o pmc -- python3 $R/bench.py --steps 3 --warmup 1 --cpu-baseline 0 --row-share 0 > /dev/null 2> $OUT/pmc_write.err) || { echo "pmc write failed"; exit 1; }
    FC=$(find $OUT/pmc_fetch -name '*counter_collection.csv' | head -1); WC=$(find $OUT/pmc_write -name '*counter_collection.csv' | head -1)
    (cd $R && python3 tools/collect_pmc.py "$FC" "$WC" $R/profiles/pmc_summary.json $TAG > /dev/null && cp $R/profiles/pmc_summary.json $OUT/pmc_summary_wavefront.json) || { echo "pmc summary failed"; exit 1; } ;;
  calib)
    for c in FETCH_SIZE WRITE_SIZE "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"; do
      d=$(echo $c | cut -d' ' -f1)
      (cd /tmp && step 60 rocprofv3 --pmc $c --output-format csv -d $OUT/calib_$d -o c -- $R/tools/micro/pmc_calib > $OUT/calib_$d.log 2>&1) || { echo "calib $c failed"; tail -5 $OUT/calib_$d.log; exit 1; }
    done ;;
  l1)
    # L1 (TCP) tag accesses and misses to L2 with their latency, L2 hits / misses: the traversal's data
    # locality on the bench frame (one pass: 4 TCP + 2 TCC counters)
    (cd /tmp && step 120 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/l1 -o l1 -- python3 $R/tools/render_once.py 0 2 > $OUT/l1.log 2>&1) || { echo "l1 pass failed"; tail -5 $OUT/l1.log; exit 1; } ;;
  l1mesh)
    # the same L1 / L2 pass over two C5-shaped mesh frames (16 spp, depth 50), plus the box's counter list
    (cd /tmp && timeout -s KILL 90 rocprofv3 -L > $OUT/counters.txt 2>&1) || echo "counter list failed (ignored)"
    (cd /tmp && step 180 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/l1m -o l1 -- python3 $R/tools/render_once.py 0 2 mesh_scene 16 50 > $OUT/l1m.log 2>&1) || { echo "l1 mesh pass failed"; tail -5 $OUT/l1m.log; exit 1; } ;;
  mix)
    # MIXSCENES="name spp depth;...": the scenes (default the bench frame, C4's and C5's)
    IFS=';' read -ra MSC <<< "${MIXSCENES:-rtow 64 8;quadric_sdl 16 50;mesh_scene 16 50}"
    for sc in "${MSC[@]}"; do
      set -- $sc
      (cd $R && bash tools/pmc_mix.sh $OUT/mix_$1 - $1 $2 $3 > $OUT/mix_$1.log 2>&1) || { echo "pmc mix $1 failed"; tail -5 $OUT/mix_$1.log; exit 1; }
      (cd /tmp && step 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/mixtr_$1 -o tr -- python3 $R/tools/render_once.py 0 2 $1 $2 $3 > $OUT/mixtr_$1.log 2>&1) || { echo "mix trace $1 failed"; exit 1; }
      (cd $R && python3 tools/valu_roofline.py $OUT/mix_$1 $(ls $OUT/mixtr_$1/*kernel_trace.csv) $OUT/valu_$1.json > $OUT/valu_$1.txt 2>&1)
    done ;;
  scenes)
    (cd /tmp && step 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/tr_c4 -o tr -- python3 $R/tools/time_scene.py default quadric 16 50 1024x1024 > $OUT/tr_c4.log 2>&1) || { echo "c4 trace failed"; tail -5 $OUT/tr_c4.log; exit 1; }
    (cd /tmp && step 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/tr_c5 -o tr -- python3 $R/tools/time_scene.py default mesh 16 50 1920x1080 > $OUT/tr_c5.log 2>&1) || { echo "c5 trace failed"; tail -5 $OUT/tr_c5.log; exit 1; } ;;
  ab)
    # this tree's bench line against the baseline worktree base/ (tools/ab_base.sh), 3 rounds interleaved
    for rep in 1 2 3; do
      (cd $R/base && step 240 python3 bench.py --cpu-baseline 0 --steps 20 --warmup 5 > $OUT/ab_base_$rep.json 2> $OUT/ab_base.err) || { echo "base bench failed"; tail -5 $OUT/ab_base.err; exit 1; }
      (cd $R && step 240 python3 bench.py --cpu-baseline 0 --steps 20 --warmup 5 > $OUT/ab_new_$rep.json 2> $OUT/ab_new.err) || { echo "bench failed"; tail -5 $OUT/ab_new.err; exit 1; }
    done
    (cd $R && python3 tools/ab_report.py $OUT/ab_base_*.json -- $OUT/ab_new_*.json | tee $OUT/ab.txt) ;;
  variants)
    # bench.py of base/, this tree's product and every dev variant (raysnail_amd/lib/var_*.so, tools/build_variant.sh),
    # 2 rounds interleaved; frames of the variants are not checked here (dev bounds may be wrong on purpose)
    B="--cpu-baseline 0 --steps 20 --warmup 5"
    for rep in 1 2; do
      if [ -d $R/base ]; then
        (cd $R/base && step 240 python3 bench.py $B > $OUT/v_base_$rep.json 2> $OUT/v.err) || { echo "base bench failed"; tail -5 $OUT/v.err; exit 1; }
      fi
      (cd $R && step 240 python3 bench.py $B > $OUT/v_prod_$rep.json 2> $OUT/v.err) || { echo "bench failed"; tail -5 $OUT/v.err; exit 1; }
      for v in $R/raysnail_amd/lib/var_*.so; do
        [ -e "$v" ] || continue
        n=$(basename $v .so)
        (cd $R && RS_HIP_LIB=$v step 240 python3 bench.py $B > $OUT/v_${n}_$rep.json 2> $OUT/v.err) || { echo "$n bench failed"; tail -5 $OUT/v.err; exit 1; }
      done
      # DEVCFGS="KNOB=v,KNOB=v;KNOB=v": dev-library configurations (rs_host.cpp RS_DEV_KNOBS), one per ';'
      IFS=';' read -ra CFGS <<< "${DEVCFGS:-}"
      for cfg in "${CFGS[@]}"; do
        n=dev_$(echo $cfg | tr ',=' '__')
        (cd $R && env RS_HIP_LIB=$R/raysnail_amd/lib/libraysnail_hip_dev.so $(echo $cfg | tr ',' ' ') timeout -k 10 240 python3 bench.py $B > $OUT/v_${n}_$rep.json 2> $OUT/v.err) || { echo "$n bench failed"; tail -5 $OUT/v.err; exit 1; }
      done
    done
    (cd $R && python3 tools/ab_report.py $OUT/v_*.json | tee $OUT/variants.txt) ;;
  travstats)
    # node steps / leaf tests per ray and per wave by ray category (a -DRS_TRAV_STATS build renamed to
    # raysnail_amd/lib/trav_stats.so: tools/build_variant.sh stats -DRS_TRAV_STATS)
    (cd $R && step 300 python3 tools/trav_stats.py $R/raysnail_amd/lib/trav_stats.so rtow,example,quadric,mesh > $OUT/trav_stats.txt 2>&1) || { echo "trav stats failed"; tail -5 $OUT/trav_stats.txt; exit 1; }
    cat $OUT/trav_stats.txt ;;
  pool)
    # C3 / C4-shaped frames with the dev library at several streaming pool sizes (RS_POOL_PATHS): iterations vs launch size
    for pp in 67108864 134217728 268435456; do
      for sc in "rtow 256 50 1920x1080" "quadric 64 50 1024x1024"; do
        (cd $R && RS_HIP_LIB=$R/raysnail_amd/lib/libraysnail_hip_dev.so RS_POOL_PATHS=$pp step 300 python3 tools/time_scene.py $R/raysnail_amd/lib/libraysnail_hip_dev.so $sc >> $OUT/pool.jsonl 2>> $OUT/pool.err) || { echo "pool $pp $sc failed"; tail -5 $OUT/pool.err; exit 1; }
        echo "pool $pp: $(tail -1 $OUT/pool.jsonl)"
      done
    done ;;
  c4)
    # C4-shaped frames (quadric.sdl + Cornell emitter 1024x1024, 64 spp, depth 50) with the product and every variant
    for v in $R/raysnail_amd/lib/libraysnail_hip.so $R/raysnail_amd/lib/var_*.so; do
      [ -e "$v" ] || continue
      (cd $R && step 300 python3 tools/time_scene.py $v quadric 64 50 1024x1024 >> $OUT/c4.jsonl 2>> $OUT/c4.err) || { echo "c4 $v failed"; tail -5 $OUT/c4.err; exit 1; }
      echo "c4: $(tail -1 $OUT/c4.jsonl)"
    done ;;
  c5)
    # C5-shaped frames (the 72k-triangle mesh scene 1920x1080, 16 spp, depth 50) with the product and every variant
    for v in $R/raysnail_amd/lib/libraysnail_hip.so $R/raysnail_amd/lib/var_*.so; do
      [ -e "$v" ] || continue
      (cd $R && step 300 python3 tools/time_scene.py $v mesh 16 50 1920x1080 >> $OUT/c5.jsonl 2>> $OUT/c5.err) || { echo "c5 $v failed"; tail -5 $OUT/c5.err; exit 1; }
      echo "c5: $(tail -1 $OUT/c5.jsonl)"
    done ;;
  c5trace)
    # kernel traces of one C5-shaped mesh frame per library (product and variants): per-launch extend / shade times
    for v in $R/raysnail_amd/lib/libraysnail_hip.so $R/raysnail_amd/lib/var_*.so; do
      [ -e "$v" ] || continue
      n=$(basename $v .so)
      (cd /tmp && step 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/c5t_$n -o tr -- python3 $R/tools/time_scene.py $v mesh 16 50 1920x1080 > $OUT/c5t_$n.log 2>&1) || { echo "c5 trace $n failed"; tail -5 $OUT/c5t_$n.log; exit 1; }
      echo "== $n" >> $OUT/c5trace.txt
      (cd $R && python3 tools/launch_times.py $OUT/c5t_$n/tr_kernel_trace.csv >> $OUT/c5trace.txt)
    done
    cat $OUT/c5trace.txt ;;
  probe)
    # kernel traces of one bench frame per library (product and variants): the first launches of each kernel
    for v in $R/raysnail_amd/lib/libraysnail_hip.so $R/raysnail_amd/lib/var_*.so; do
      [ -e "$v" ] || continue
      n=$(basename $v .so)
      (cd /tmp && RS_HIP_LIB=$v step 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/pr_$n -o tr -- python3 $R/tools/render_once.py 0 1 > $OUT/pr_$n.log 2>&1) || { echo "probe trace $n failed"; tail -5 $OUT/pr_$n.log; exit 1; }
      echo "== $n" >> $OUT/probe.txt
      (cd $R && python3 tools/launch_times.py $OUT/pr_$n/tr_kernel_trace.csv 20 first >> $OUT/probe.txt)
    done
    cat $OUT/probe.txt ;;
  c4trace)
    # kernel trace of C4-shaped frames (quadric.sdl + Cornell emitter 1024x1024, 256 spp, depth 50)
    (cd /tmp && step 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c4t -o tr -- python3 $R/tools/time_scene.py default quadric 256 50 1024x1024 > $OUT/c4t.log 2>&1) || { echo "c4 trace failed"; tail -5 $OUT/c4t.log; exit 1; }
    tail -1 $OUT/c4t.log ;;
  c3)
    # C3-shaped frames (RTIOW 1920x1080, 64 spp, depth 50) with the product, every variant, and the dev library
    # with RS_EXT_SPLIT=1 (carried part and camera part in separate launches on iterations with both)
    for v in $R/raysnail_amd/lib/libraysnail_hip.so $R/raysnail_amd/lib/var_*.so; do
      [ -e "$v" ] || continue
      (cd $R && step 300 python3 tools/time_scene.py $v rtow 64 50 1920x1080 >> $OUT/c3.jsonl 2>> $OUT/c3.err) || { echo "c3 $v failed"; tail -5 $OUT/c3.err; exit 1; }
      echo "c3: $(tail -1 $OUT/c3.jsonl)"
    done
    (cd $R && RS_HIP_LIB=$R/raysnail_amd/lib/libraysnail_hip_dev.so RS_EXT_SPLIT=1 step 300 python3 tools/time_scene.py $R/raysnail_amd/lib/libraysnail_hip_dev.so rtow 64 50 1920x1080 >> $OUT/c3.jsonl 2>> $OUT/c3.err) || { echo "c3 dev split failed"; exit 1; }
    echo "c3 dev RS_EXT_SPLIT=1: $(tail -1 $OUT/c3.jsonl)" ;;
  c2)
    # C2-shaped frames (example.sdl 800x500, 64 spp, depth 50) with the product and every variant
    for v in $R/raysnail_amd/lib/libraysnail_hip.so $R/raysnail_amd/lib/var_*.so; do
      [ -e "$v" ] || continue
      (cd $R && step 300 python3 tools/time_scene.py $v example 64 50 800x500 >> $OUT/c2.jsonl 2>> $OUT/c2.err) || { echo "c2 $v failed"; tail -5 $OUT/c2.err; exit 1; }
      echo "c2: $(tail -1 $OUT/c2.jsonl)"
    done ;;
  benchprof)
    # bench.py itself under rocprofv3 --kernel-trace --stats (the contract's "same command"): its bench line and the
    # kernel statistics, whose k_wfs_extend average the line's event-timed avg_launch_ms should agree with
    (cd /tmp && step 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/benchprof -o bp -- python3 $R/bench.py --cpu-baseline 0 --row-share 0 > $OUT/bench_under_rocprof.json 2> $OUT/benchprof.err) || { echo "bench under rocprof failed"; tail -5 $OUT/benchprof.err; exit 1; }
    tail -1 $OUT/bench_under_rocprof.json
    # the line's roofline recomputed from the trace's statistics-frame launches (tools/trace_roofline.py)
    (cd $R && python3 tools/trace_roofline.py $OUT/benchprof/bp_kernel_trace.csv $OUT/bench_under_rocprof.json | tee $OUT/trace_roofline.json) ;;
  meshtests)
    (cd $R && step 600 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu -k "mesh or c5 or C5 or million" > $OUT/pytest_mesh.log 2>&1) || { echo "mesh tests failed"; tail -30 $OUT/pytest_mesh.log; exit 1; }
    tail -1 $OUT/pytest_mesh.log ;;
  finish)
    # depth-50 frames with the dev library at several finish points (RS_FINISH_AFTER: wavefront iterations after the
    # last injection before k_wfs_finish; 0 = none): C2, a C3-shaped RTIOW frame, C4-shaped quadric frames
    for fa in ${FINISH_AFTER:-0 4 8 12}; do
      for sc in "example 64 50 800x500" "rtow 64 50 1920x1080" "quadric 64 50 1024x1024"; do
        (cd $R && RS_HIP_LIB=$R/raysnail_amd/lib/libraysnail_hip_dev.so RS_FINISH_AFTER=$fa step 300 python3 tools/time_scene.py $R/raysnail_amd/lib/libraysnail_hip_dev.so $sc >> $OUT/finish.jsonl 2>> $OUT/finish.err) || { echo "finish $fa $sc failed"; tail -5 $OUT/finish.err; exit 1; }
        echo "finish_after $fa: $(tail -1 $OUT/finish.jsonl)"
      done
    done ;;
  abtrace)
    # kernel traces of the bench frames (tools/render_once.py, 5 frames): the baseline worktree base/, then this tree
    (cd /tmp && step 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/abt_base -o t -- python3 $R/base/tools/render_once.py 0 5 > $OUT/abt_base.log 2>&1) || { echo "base trace failed"; exit 1; }
    (cd /tmp && step 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/abt_new -o t -- python3 $R/tools/render_once.py 0 5 > $OUT/abt_new.log 2>&1) || { echo "trace failed"; exit 1; }
    (cd $R && python3 tools/trace_cmp.py $OUT/abt_base/t_kernel_trace.csv $OUT/abt_new/t_kernel_trace.csv | tee $OUT/abtrace.txt) ;;
  iters)
    # one lane, the dev library: per-iteration queue counts (RS_DUMP_ITERS) under a kernel trace; then the
    # per-iteration table (extend and shading launch times)
    # ITERSCENES="name spp depth;...": the frames (default the bench frame and C2's example.sdl frame)
    IFS=';' read -ra ISC <<< "${ITERSCENES:-rtow 64 8;example_sdl 64 50}"
    for sc in "${ISC[@]}"; do
      set -- $sc
      (cd /tmp && RS_HIP_LIB=$R/raysnail_amd/lib/libraysnail_hip_dev.so RS_DUMP_ITERS=1 step 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/iters_$1 -o it -- python3 $R/tools/render_once.py 0 4 $1 $2 $3 > $OUT/iters_$1.log 2>&1) || { echo "iters trace $1 failed"; tail -5 $OUT/iters_$1.log; exit 1; }
      (cd $R && python3 tools/iter_table.py $OUT/iters_$1.log $(ls $OUT/iters_$1/*kernel_trace.csv) | tee $OUT/iters_$1.txt)
    done ;;
  passtest)
    (cd $R && step 600 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu -k "passes or streaming_pool or queue_counter" > $OUT/pytest_passes.log 2>&1) || { echo "passes tests failed"; tail -30 $OUT/pytest_passes.log; exit 1; }
    tail -1 $OUT/pytest_passes.log ;;
  passes)
    # rs_render_device_passes (K passes as one sample stream) against K pipelined one-pass frames: bench frame, N = 8 share
    # PASSARGS="...;...": one probe run per entry (default the bench frame and its N = 8 share)
    IFS=';' read -ra PA <<< "${PASSARGS:- }"
    for a in "${PA[@]}"; do
      (cd $R && step 300 python3 tools/passes_probe.py $a >> $OUT/passes.jsonl 2>> $OUT/passes.err) || { echo "passes probe failed"; tail -5 $OUT/passes.err; exit 1; }
    done
    cat $OUT/passes.jsonl ;;
  passtrace)
    # kernel traces of K = 12 row-share frames, one call per pass against the passes stream (one lane, one slot)
    for m in single stream; do
      (cd /tmp && step 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/pt_$m -o t -- python3 $R/tools/passes_trace.py $m 12 ${PT_ROWSTEP:-8} > $OUT/pt_$m.log 2>&1) || { echo "passes trace $m failed"; tail -5 $OUT/pt_$m.log; exit 1; }
      (cd $R && echo "== $m" >> $OUT/passtrace.txt && python3 tools/trace_sum.py $(ls $OUT/pt_$m/*kernel_trace.csv) 12 >> $OUT/passtrace.txt)
    done
    cat $OUT/passtrace.txt ;;
  abenv)
    # this build's bench line against the dev library with ABENV (a dev knob that turns a feature off), 3 rounds
    B="--cpu-baseline 0 --steps 20 --warmup 5"
    for rep in 1 2 3; do
      (cd $R && step 240 env RS_HIP_LIB=$R/raysnail_amd/lib/libraysnail_hip_dev.so $ABENV python3 bench.py $B > $OUT/abenv_off_$rep.json 2> $OUT/abenv.err) || { echo "dev bench failed"; tail -5 $OUT/abenv.err; exit 1; }
      (cd $R && step 240 python3 bench.py $B > $OUT/abenv_on_$rep.json 2> $OUT/abenv.err) || { echo "bench failed"; tail -5 $OUT/abenv.err; exit 1; }
    done
    (cd $R && python3 tools/ab_report.py $OUT/abenv_off_*.json -- $OUT/abenv_on_*.json | tee $OUT/abenv.txt) ;;
  envtrace)
    # kernel traces of 4 bench frames (tools/render_once.py): the dev library with ABENV, then this build; per-kernel
    # time per frame of the last two (tools/trace_sum.py)
    (cd /tmp && step 200 env RS_HIP_LIB=$R/raysnail_amd/lib/libraysnail_hip_dev.so $ABENV rocprofv3 --kernel-trace --output-format csv -d $OUT/et_off -o t -- python3 $R/tools/render_once.py 0 4 > $OUT/et_off.log 2>&1) || { echo "env trace failed"; tail -5 $OUT/et_off.log; exit 1; }
    (cd /tmp && step 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/et_on -o t -- python3 $R/tools/render_once.py 0 4 > $OUT/et_on.log 2>&1) || { echo "trace failed"; tail -5 $OUT/et_on.log; exit 1; }
    for m in off on; do (cd $R && echo "== $m" >> $OUT/envtrace.txt && python3 tools/trace_sum.py $(ls $OUT/et_$m/*kernel_trace.csv) 2 >> $OUT/envtrace.txt); done
    cat $OUT/envtrace.txt ;;
  libtrace)
    # kernel traces of 4 bench frames (tools/render_once.py) with the product and every variant; per-kernel time per
    # frame of the last two (tools/trace_sum.py)
    for v in $R/raysnail_amd/lib/libraysnail_hip.so $R/raysnail_amd/lib/var_*.so; do
      [ -e "$v" ] || continue
      n=$(basename $v .so)
      (cd /tmp && RS_HIP_LIB=$v step 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/lt_$n -o t -- python3 $R/tools/render_once.py 0 4 > $OUT/lt_$n.log 2>&1) || { echo "lib trace $n failed"; tail -5 $OUT/lt_$n.log; exit 1; }
      (cd $R && echo "== $n" >> $OUT/libtrace.txt && python3 tools/trace_sum.py $(ls $OUT/lt_$n/*kernel_trace.csv) 2 >> $OUT/libtrace.txt)
    done
    cat $OUT/libtrace.txt ;;
  splitab)
    # the streaming extend in two launches on iterations with carried paths and camera samples (dev RS_EXT_SPLIT=1)
    # against the product: C2-, C3-shaped frames and the C5-like small rtow frame, 2 rounds
    for rep in 1 2; do
      for sc in "example 64 50 800x500" "rtow 64 50 1920x1080" "rtow 16 50 800x500"; do
        (cd $R && step 300 python3 tools/time_scene.py $R/raysnail_amd/lib/libraysnail_hip.so $sc >> $OUT/splitab.jsonl 2>> $OUT/splitab.err) || { echo "split ab failed"; tail -5 $OUT/splitab.err; exit 1; }
        (cd $R && RS_HIP_LIB=$R/raysnail_amd/lib/libraysnail_hip_dev.so RS_EXT_SPLIT=1 step 300 python3 tools/time_scene.py $R/raysnail_amd/lib/libraysnail_hip_dev.so $sc >> $OUT/splitab.jsonl 2>> $OUT/splitab.err) || { echo "split ab dev failed"; exit 1; }
      done
    done
    cat $OUT/splitab.jsonl ;;
  configs)
    (cd $R && step 900 python3 tools/bench_configs.py > $OUT/configs.jsonl 2> $OUT/configs.err) || { echo "config sweep failed"; tail -5 $OUT/configs.err; exit 1; }
    cat $OUT/configs.jsonl ;;
  *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo done
