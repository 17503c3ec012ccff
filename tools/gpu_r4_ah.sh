#!/bin/bash
# round 4, call AH: bench.py on its own non-default stream -- the default bench line (value unchanged?)
# and the 2-rank gloo rehearsal of the N > 1 line (execute_ms should now bracket the pass)
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r4ah_bench.log 2>&1 || exit $?
bash tools/gpu_multirank_rehearsal.sh r04ah
