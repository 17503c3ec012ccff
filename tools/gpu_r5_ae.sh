#!/bin/bash
# round 5, call AE: the three-TU library (tap_launch.hip on the default scheduler, tap_f32.hip on
# iterative-maxocc) against the two-TU base, then the final validation (tools/gpu_r5_final.sh)
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V=dpe-mvs_amd/lib/variants
AB_ROUNDS=3 timeout -k 10 400 python -u tools/ab_libs.py $V/tap_base.so dpe-mvs_amd/lib/libdpe_mvs.so > gpurun_out/r05ae_ab_split.log 2>&1 || exit $?
bash tools/gpu_r5_final.sh ${1:-r05ae}
