#!/bin/bash
# round 4, call P: RANSAC edge walks stopped at the first crossing (DPE_GN_RSC) and the wave-shared
# probe walks (DPE_GN_COOP, 2 lines) on the pixel-first default -- A/B, parity, slowest waves
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V=dpe-mvs_amd/lib/variants
AB_ROUNDS=5 timeout -k 10 500 python -u tools/ab_libs.py dpe-mvs_amd/lib/libdpe_mvs.so $V/rsc.so $V/c2.so $V/rscc2.so $V/head.so > gpurun_out/r4p_ab.log 2>&1 || exit $?
DPE_MVS_LIB=$PWD/$V/rscc2.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4p_parity.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/gn_times.py $V/gntrsc.so > gpurun_out/r4p_gn_times_rsc.log 2>&1
