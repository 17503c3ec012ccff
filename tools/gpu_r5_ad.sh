#!/bin/bash
# round 5, call AD: LLVM scheduler of the tap translation unit (strong sweep, DepthToWeak, LocalRefine,
# init): iterative-maxocc (base) / default / max-occupancy-experimental
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V=dpe-mvs_amd/lib/variants
AB_ROUNDS=4 timeout -k 10 500 python -u tools/ab_libs.py $V/tap_base.so $V/tap_def.so $V/tap_exp.so > gpurun_out/r05ad_ab_tapsched.log 2>&1
