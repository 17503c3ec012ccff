#!/bin/bash
# round 5, call D: forms of the rare slow tap loop under restatement choice 8 -- interleaved timing
# A/B (round-4 Newton build, row loop, exponent flag + redo, rolled generic loop, and an inexact
# IEEE-slow-path bound) and the slow-patch share from the pool statistics build
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V=dpe-mvs_amd/lib/variants
timeout -k 10 200 python -u tools/pool_stats.py $V/pstat.so > gpurun_out/r05d_pool_stats.log 2>&1 || exit $?
AB_NOCHECK=1 AB_ROUNDS=4 timeout -k 10 600 python -u tools/ab_libs.py $V/newton.so $V/rcp_s1.so $V/rcp_s2.so $V/rcp_s3.so $V/ieee_bound.so > gpurun_out/r05d_ab_slow.log 2>&1
