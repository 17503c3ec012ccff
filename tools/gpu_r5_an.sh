#!/bin/bash
# round 5, call AN: waves per workgroup of DepthToWeak (2 / 8 against 4) and of the strong sweep
# (2 / 8 against 4)
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V=dpe-mvs_amd/lib/variants
AB_ROUNDS=3 timeout -k 10 700 python -u tools/ab_libs.py $V/base.so $V/d2.so $V/d8.so $V/s2.so $V/s8.so > gpurun_out/r05an_ab_wgsize.log 2>&1
