#!/bin/bash
# round 5, call AL: the main unit (SLP vectorizer off) under the default scheduler against
# gcn-iterative-max-occupancy-experimental and max-memory-clause
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V=dpe-mvs_amd/lib/variants
AB_ROUNDS=3 timeout -k 10 500 python -u tools/ab_libs.py $V/base.so $V/m_exp.so $V/m_mc.so > gpurun_out/r05al_ab_mainsched.log 2>&1
