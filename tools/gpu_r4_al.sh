#!/bin/bash
# round 4, call AL: LLVM scheduler strategies for the tap kernels' translation unit and for both
# (iterative-minreg, max-ilp) against the default build (iterative-maxocc tap TU) -- A/B, identical outputs
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V=dpe-mvs_amd/lib/variants
AB_ROUNDS=5 timeout -k 10 600 python -u tools/ab_libs.py dpe-mvs_amd/lib/libdpe_mvs.so $V/tap_minreg.so $V/tap_maxilp.so $V/all_minreg.so $V/all_maxilp.so > gpurun_out/r4al_ab.log 2>&1
