#!/bin/bash
# round 4, call X: the weak sweep with the neighbour loop's dead patch sides removed (DPE_WEAK_NBMAX),
# with and without the zero-scratch field copies
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V=dpe-mvs_amd/lib/variants
AB_ROUNDS=5 timeout -k 10 500 python -u tools/ab_libs.py dpe-mvs_amd/lib/libdpe_mvs.so $V/nbmax.so $V/nbz.so $V/zscr.so > gpurun_out/r4x_ab.log 2>&1
