#!/bin/bash
# round 5, call AA: DepthToWeak at 5 waves per SIMD (96 VGPRs, 104 B/lane scratch) against 4
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V=dpe-mvs_amd/lib/variants
AB_ROUNDS=4 timeout -k 10 500 python -u tools/ab_libs.py $V/d4.so $V/d5.so > gpurun_out/r05aa_ab_d2w5.log 2>&1
