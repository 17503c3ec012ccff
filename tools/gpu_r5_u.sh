#!/bin/bash
# round 5, call U: pool statistics incl. how often a weak pixel's current / fit plane is one of its
# candidate planes
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/pool_stats.py dpe-mvs_amd/lib/variants/pstat.so > gpurun_out/r05u_pool_stats.log 2>&1
