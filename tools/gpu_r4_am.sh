#!/bin/bash
# round 4, call AM: scheduler options beside the strategy -- AMDGPU register-pressure trackers (tap
# unit / both units), the default scheduler's metric bias 0 and no high-RP reschedule stage -- A/B
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V=dpe-mvs_amd/lib/variants
AB_ROUNDS=5 timeout -k 10 600 python -u tools/ab_libs.py dpe-mvs_amd/lib/libdpe_mvs.so $V/tap_trk.so $V/both_trk.so $V/bias0.so $V/nohirp.so > gpurun_out/r4am_ab.log 2>&1
