#!/bin/bash
# round 4, call W: the full -m gpu suite and smoke on the final build
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
bash tools/gpu_round2_a.sh r04w || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > gpurun_out/r04w_smoke.log 2>&1
