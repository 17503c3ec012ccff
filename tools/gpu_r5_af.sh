#!/bin/bash
# round 5, call AF: the 8-bit / quarter-integer tap unit under the default scheduler (base) against
# max-ilp, max-memory-clause and iterative-minreg (all four without scratch since choice 8)
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V=dpe-mvs_amd/lib/variants
AB_ROUNDS=3 timeout -k 10 500 python -u tools/ab_libs.py $V/s_def.so $V/s_ilp.so $V/s_mc.so $V/s_mr.so > gpurun_out/r05af_ab_sched2.log 2>&1
