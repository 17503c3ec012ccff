#!/bin/bash
# round 4, call F: GenNeighbours per-pixel work counts and wave lifetimes (-DDPE_GN_TIMES=1 build)
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/gn_times.py dpe-mvs_amd/lib/variants/gntimes.so > gpurun_out/r04f_gn_times.log 2>&1
