#!/bin/bash
# round 3 GPU call D: gather locality of two line-statistics builds
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
for lib in "$@"; do
  echo "== $lib" >> gpurun_out/r3d_lines.log
  timeout -k 10 300 python -u tools/line_stats.py "$lib" >> gpurun_out/r3d_lines.log 2>&1 || exit $?
done
