#!/bin/bash
# round 4, call V: the final build's one-stream kernel trace + stats of the bench command, then the
# PMC traffic passes (tools/pmc.sh) -- profiles/r04f_*
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
DPE_OVERLAP=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/r04f_prof" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 2 --no-e2e --no-cpu-baseline --no-pass-types --no-pipeline > "$GRAFT_REPO_ROOT/gpurun_out/r04f_prof_bench.log" 2>&1 || exit $?
cd "$GRAFT_REPO_ROOT"
bash tools/pmc.sh r04f > gpurun_out/r04f_pmc.log 2>&1
