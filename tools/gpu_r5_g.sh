#!/bin/bash
# round 5, call G: the final build's one-stream kernel trace + stats (DPE_OVERLAP=0) and its
# overlapped-pass timeline (bench on its own stream)
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
tag=r05g
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/${tag}_tl" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --no-instrument > "$GRAFT_REPO_ROOT/gpurun_out/${tag}_tl_bench.log" 2>&1 || exit $?
DPE_OVERLAP=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/${tag}_prof" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 2 --no-e2e --no-cpu-baseline --no-pass-types --no-pipeline > "$GRAFT_REPO_ROOT/gpurun_out/${tag}_prof_bench.log" 2>&1
