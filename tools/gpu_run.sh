#!/bin/bash
# The one GPU-box runner (replaces rounds 2-5's one-off lease scripts).  Run through gpurun:
#   gpurun --timeout 1200 -- bash tools/gpu_run.sh TAG STEP [STEP ...]
# Steps run in order, each under its own time limit; the first failing step ends the call (no GPU
# step runs after a fault, abort or time-out).  Logs go to gpurun_out/TAG_<step>.log.
#   tests        the -m gpu suite                            subset:<pytest args>  a part of it
#   smoke        __graft_entry__.smoke()                     bench        the default bench line (20 steps)
#   quick        bench without the side lines (10 steps)     prof         one-stream rocprofv3 kernel trace + stats
#   timeline     overlapped kernel trace (tools/timeline.py) pmc          PMC traffic + bottleneck passes
#   rehearsal    `bench.py --gpus 2` over gloo on one GPU    ab:<a.so,b.so,...>  interleaved A/B (tools/ab_libs.py)
#   phase:<so>   phase profile of a DPE_DIAG build
#   run:<cmd>    any command (quote the step: "run:DPE_DBG_GN_ONCE=1 python -u tools/gn_ceiling.py 10")
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
tag=$1; shift
[ -n "$tag" ] || { echo "usage: gpu_run.sh TAG STEP..."; exit 2; }
nrun=0
PT="python -u -m pytest -p no:cacheprovider --timeout 900 --timeout-method thread"
for step in "$@"; do
  name=${step%%:*}; arg=${step#*:}; [ "$arg" = "$step" ] && arg=
  log=$R/gpurun_out/${tag}_${name}.log
  echo "== $step ($(date +%T))"
  case $name in
    tests)  (cd "$R" && timeout -k 10 1100 $PT tests -m gpu -v --durations=15 > "$log" 2>&1) ;;
    subset) (cd "$R" && timeout -k 10 900 $PT $arg -m gpu -v --durations=10 > "$log" 2>&1) ;;
    smoke)  (cd "$R" && timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > "$log" 2>&1) ;;
    bench)  (cd "$R" && timeout -k 10 700 python -u bench.py --steps 20 --warmup 5 > "$log" 2>&1) ;;
    quick)  (cd "$R" && timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-e2e --no-cpu-baseline \
               --no-pass-types --no-pipeline > "$log" 2>&1) ;;
    prof)   (cd /tmp && export TMPDIR=/tmp && DPE_OVERLAP=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats \
               --output-format csv -d "$R/gpurun_out/${tag}_prof" -o run -- python3 "$R/bench.py" --steps 10 --warmup 2 \
               --no-e2e --no-cpu-baseline --no-pass-types --no-pipeline > "$log" 2>&1) ;;
    timeline) (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv \
               -d "$R/gpurun_out/${tag}_tl" -o run -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-instrument \
               > "$log" 2>&1) ;;
    pmc)    (cd "$R" && bash tools/pmc.sh "$tag" > "$log" 2>&1 && bash tools/pmc_bottleneck.sh "$tag" >> "$log" 2>&1) ;;
    rehearsal) (cd "$R" && DPE_BENCH_BACKEND=gloo timeout -k 10 500 python -u bench.py --gpus 2 --steps 3 --warmup 1 \
               --no-pass-types --no-config5 > "$log" 2>&1) ;;
    ab)     (cd "$R" && AB_ROUNDS=${AB_ROUNDS:-5} timeout -k 10 600 python -u tools/ab_libs.py ${arg//,/ } > "$log" 2>&1) ;;
    phase)  (cd "$R" && timeout -k 10 200 python -u tools/phase_prof.py "$arg" > "$log" 2>&1) ;;
    run)    log=$R/gpurun_out/${tag}_run$((++nrun)).log
            (cd "$R" && timeout -k 10 400 env $arg > "$log" 2>&1) ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
  rc=$?
  echo "$step rc=$rc" | tee -a "$log"
  [ $rc -eq 0 ] || exit $rc
done
echo "GPU_RUN_DONE $tag"
