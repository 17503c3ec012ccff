#!/bin/bash
# round 3 GPU call G: bit-checked A/B of variant libraries + gather statistics of a line-stats build
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
lstat=$1; shift
AB_ROUNDS=4 timeout -k 10 500 python -u tools/ab_libs.py "$@" > gpurun_out/${TAG}_ab.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/line_stats.py "$lstat" > gpurun_out/${TAG}_lines.log 2>&1
