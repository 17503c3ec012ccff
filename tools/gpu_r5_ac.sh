#!/bin/bash
# round 5, call AC: LLVM scheduler strategies for the main translation unit (weak sweep, GenNeighbours,
# RANSAC, lists) after the round's changes -- interleaved A/B with output check
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V=dpe-mvs_amd/lib/variants
AB_ROUNDS=4 timeout -k 10 500 python -u tools/ab_libs.py $V/sch_default.so $V/sch_iterative-maxocc.so $V/sch_gcn-iterative-max-occupancy-experimental.so > gpurun_out/r05ac_ab_sched.log 2>&1
