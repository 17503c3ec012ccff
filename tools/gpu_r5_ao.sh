#!/bin/bash
# round 5, call AO: DepthToWeak at 2 / 1 waves per workgroup combined with the strong sweep at 2
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V=dpe-mvs_amd/lib/variants
AB_ROUNDS=3 timeout -k 10 700 python -u tools/ab_libs.py $V/base.so $V/d2.so $V/d2s2.so $V/d1s2.so $V/d1.so > gpurun_out/r05ao_ab_wgsize2.log 2>&1
