#!/bin/bash
# round 3 GPU call J: bit-identity + timing A/B of variant libraries, then the weak-sweep path
# statistics of a -DDPE_WEAK_STATS=1 build (last argument)
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
tag=${TAG:-r3j}
stats=${@: -1}
libs=("${@:1:$#-1}")
AB_ROUNDS=${AB_ROUNDS:-4} timeout -k 10 500 python -u tools/ab_libs.py "${libs[@]}" > gpurun_out/${tag}_ab.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/weak_stats.py $stats > gpurun_out/${tag}_wstat.log 2>&1
