#!/bin/bash
# round 4, call AD: per-colour RANSAC fits on the two weak-sweep streams (DPE_RANSAC_SPLIT) against
# the new default (two-stream weak sweeps) -- A/B and parity of both
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V=dpe-mvs_amd/lib/variants
AB_ROUNDS=6 timeout -k 10 500 python -u tools/ab_libs.py dpe-mvs_amd/lib/libdpe_mvs.so $V/rsplit.so $V/head.so > gpurun_out/r4ad_ab.log 2>&1 || exit $?
DPE_MVS_LIB=$PWD/$V/rsplit.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_resident.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r4ad_parity.log 2>&1
