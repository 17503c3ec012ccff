#!/bin/bash
# round 4, call K: the weak sweep's register / scratch trade-off (T copies, pass-constant patch
# parameters) against the committed build, interleaved
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V=dpe-mvs_amd/lib/variants
AB_ROUNDS=4 timeout -k 10 500 python -u tools/ab_libs.py dpe-mvs_amd/lib/libdpe_mvs.so $V/head.so $V/tcopy0.so $V/tpc.so $V/t0wph1.so $V/wph1.so > gpurun_out/r4k_ab.log 2>&1
