#!/bin/bash
# round 4, call N: GenNeighbours' probe walks shared by the wave (DPE_GN_COOP) -- A/B, parity of the
# cooperative build, and the slowest waves of both timing builds
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V=dpe-mvs_amd/lib/variants
AB_ROUNDS=4 timeout -k 10 500 python -u tools/ab_libs.py dpe-mvs_amd/lib/libdpe_mvs.so $V/head.so $V/coop.so $V/coopm5.so $V/coop4.so $V/coop16.so > gpurun_out/r4n_ab.log 2>&1 || exit $?
DPE_MVS_LIB=$PWD/$V/coop.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4n_parity_coop.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/gn_times.py $V/gntimes3.so > gpurun_out/r4n_gn_times.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/gn_times.py $V/gntcoop.so > gpurun_out/r4n_gn_times_coop.log 2>&1
