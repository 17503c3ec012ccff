#!/bin/bash
# round 5, final call: full -m gpu suite, smoke, bench (20 steps) and the one-stream kernel trace of
# the bench command for the committed summary
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
tag=${1:-r05z}
bash tools/gpu_round2_a.sh $tag || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > gpurun_out/${tag}_smoke.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/${tag}_bench.log 2>&1 || exit $?
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
DPE_OVERLAP=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/${tag}_prof" -o run -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-e2e --no-cpu-baseline --no-pass-types --no-pipeline > "$R/gpurun_out/${tag}_prof_bench.log" 2>&1
