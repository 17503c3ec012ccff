#!/bin/bash
# round 4, call L: weak sweep codegen A/B (round-3 register / scratch layout restored as default) and
# the Bresenham walks on 8x8 bit tiles (bres_walk.h walk_tiles), then the parity suite on the
# tiled build (DPE_MVS_LIB)
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V=dpe-mvs_amd/lib/variants
AB_ROUNDS=4 timeout -k 10 500 python -u tools/ab_libs.py dpe-mvs_amd/lib/libdpe_mvs.so $V/head.so $V/zscr.so $V/t0r1.so $V/wph1.so $V/tpc.so $V/tile4.so $V/tile4m5.so $V/tile2m5.so $V/tile8.so > gpurun_out/r4l_ab.log 2>&1 || exit $?
DPE_MVS_LIB=$PWD/$V/tile4.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4l_parity_tile4.log 2>&1
