#!/bin/bash
# round 4, call O: GenNeighbours' probe walks from the pixel first (DPE_GN_PIXFIRST) and the shared
# walks with fewer lines (DPE_GN_COOP_MAX 2 / 4) -- A/B, parity of the candidate, slowest waves
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V=dpe-mvs_amd/lib/variants
AB_ROUNDS=4 timeout -k 10 500 python -u tools/ab_libs.py dpe-mvs_amd/lib/libdpe_mvs.so $V/pixf.so $V/pixfc4.so $V/coop2.so $V/coop4.so $V/pixfc2.so > gpurun_out/r4o_ab.log 2>&1 || exit $?
DPE_MVS_LIB=$PWD/$V/pixfc4.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4o_parity.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/gn_times.py $V/gntpixf.so > gpurun_out/r4o_gn_times_pixf.log 2>&1
