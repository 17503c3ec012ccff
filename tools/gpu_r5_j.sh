#!/bin/bash
# round 5, call J: HIP stream priorities for the pass / aux streams (pre-join window), interleaved A/B
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V=dpe-mvs_amd/lib/variants
AB_ROUNDS=5 timeout -k 10 500 python -u tools/ab_libs.py $V/prio0.so $V/prio1.so $V/prio2.so > gpurun_out/r05j_ab_prio.log 2>&1
