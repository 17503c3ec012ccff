#!/bin/bash
# round 4, call AN: the packed tap loop's row unroll (DPE_UNROLL_ROWS 0 = rolled, 2, 3; default 1 = all
# six rows) -- A/B, identical outputs
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V=dpe-mvs_amd/lib/variants
AB_ROUNDS=5 timeout -k 10 600 python -u tools/ab_libs.py dpe-mvs_amd/lib/libdpe_mvs.so $V/ur0.so $V/ur2.so $V/ur3.so > gpurun_out/r4an_ab.log 2>&1
