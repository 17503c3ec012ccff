#!/bin/bash
# round 4, call U: GenNeighbours' resident waves capped by unused LDS (DPE_GN_LDS_PAD: 4 / 2.75 / 2
# waves per SIMD), alone and with the fork after RandomInitialization -- overlapped wall A/B
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V=dpe-mvs_amd/lib/variants
AB_ROUNDS=5 timeout -k 10 500 python -u tools/ab_libs.py dpe-mvs_amd/lib/libdpe_mvs.so $V/pad4.so $V/pad3.so $V/pad2.so $V/pad3ri.so $V/pad2ri.so > gpurun_out/r4u_ab.log 2>&1
