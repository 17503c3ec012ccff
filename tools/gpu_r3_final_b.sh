#!/bin/bash
# round 3 final, part B: one-stream rocprofv3 kernel trace and the PMC traffic / bottleneck passes
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
tag=${1:-r03}
cd /tmp && export TMPDIR=/tmp
DPE_OVERLAP=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/${tag}_prof" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 2 --no-e2e --no-cpu-baseline --no-pass-types --no-pipeline > "$GRAFT_REPO_ROOT/gpurun_out/${tag}_prof_bench.log" 2>&1 || exit $?
cd "$GRAFT_REPO_ROOT"
bash tools/pmc.sh $tag > gpurun_out/${tag}_pmc.log 2>&1 || exit $?
bash tools/pmc_bottleneck.sh $tag > gpurun_out/${tag}_pmcb.log 2>&1
