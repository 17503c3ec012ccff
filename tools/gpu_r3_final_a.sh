#!/bin/bash
# round 3 final, part A: the full -m gpu suite, smoke and the bench line of the in-tree build
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
tag=${1:-r03}
bash tools/gpu_round2_a.sh $tag || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > gpurun_out/${tag}_smoke.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/${tag}_bench.log 2>&1
