#!/bin/bash
# round 4, call G: A/B of the GenNeighbours probe changes (direction table + fast angle test +
# multiply modulo: gnopt; + 64-bit-product Philox: gnopt64; Philox alone: ph64), bit-identical
# outputs asserted; then the work counts of the optimised build
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V=dpe-mvs_amd/lib/variants
timeout -k 10 500 python -u tools/ab_libs.py dpe-mvs_amd/lib/libdpe_mvs.so $V/gnopt.so $V/gnopt64.so $V/ph64.so > gpurun_out/r04g_ab.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/gn_times.py $V/gntimes2.so > gpurun_out/r04g_gn_times.log 2>&1
