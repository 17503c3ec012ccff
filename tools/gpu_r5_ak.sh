#!/bin/bash
# round 5, call AK: the strong sweep at 5 waves/SIMD (96 VGPRs, 20 / 44 B/lane of scratch) against 4
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V=dpe-mvs_amd/lib/variants
AB_ROUNDS=3 timeout -k 10 400 python -u tools/ab_libs.py $V/base.so $V/s5.so > gpurun_out/r05ak_ab_strong5.log 2>&1
