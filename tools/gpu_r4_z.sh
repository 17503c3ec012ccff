#!/bin/bash
# round 4, call Z: bench line of the final default build
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r4z_bench.log 2>&1
