#!/bin/bash
# round 4, call AA: the full -m gpu suite and smoke on the final build (RANSAC over the WEAK list)
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
bash tools/gpu_round2_a.sh r04aa || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > gpurun_out/r04aa_smoke.log 2>&1
