#!/bin/bash
# round 4, call AF: overlapped timeline of the final build (two-stream weak sweeps and fits)
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/r04af_tl" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --no-instrument > "$GRAFT_REPO_ROOT/gpurun_out/r04af_tl_bench.log" 2>&1
