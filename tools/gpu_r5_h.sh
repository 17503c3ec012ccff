#!/bin/bash
# round 5, call H: GenNeighbours per-pixel / per-wave durations and work counts (DPE_DIAG=8 build)
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/gn_times.py dpe-mvs_amd/lib/variants/gnatt.so > gpurun_out/r05h_gn_attempts.log 2>&1
