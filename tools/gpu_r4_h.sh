#!/bin/bash
# round 4, call H: GPU parity of the default build, then the A/B of the GenNeighbours probe changes
# with the corrected multiply-modulo (tools/check_gn_mod.c), then the optimised build's work counts
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r4h_parity.log 2>&1 || exit $?
V=dpe-mvs_amd/lib/variants
timeout -k 10 500 python -u tools/ab_libs.py dpe-mvs_amd/lib/libdpe_mvs.so $V/dirtab.so $V/gnopt.so $V/gnopt64.so $V/ph64.so $V/wgpool.so $V/slowrows.so $V/srgpool.so > gpurun_out/r4h_ab.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/gn_times.py $V/gntimes2.so > gpurun_out/r4h_gn_times.log 2>&1
