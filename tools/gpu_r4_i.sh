#!/bin/bash
# round 4, call I: parity of the default build (weak sweep without scratch, DepthToWeak's slow tap
# loop by rows), then the A/B against the committed build and the weak sweep's phase-1 variants
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r4i_parity.log 2>&1 || exit $?
V=dpe-mvs_amd/lib/variants
AB_ROUNDS=4 timeout -k 10 500 python -u tools/ab_libs.py dpe-mvs_amd/lib/libdpe_mvs.so $V/head.so $V/d2wrow0.so $V/tbatch.so $V/srows.so $V/wph1.so > gpurun_out/r4i_ab.log 2>&1
