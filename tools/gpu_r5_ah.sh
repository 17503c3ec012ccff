#!/bin/bash
# round 5, call AH: the main unit (weak sweep, GenNeighbours, init, RANSAC) with scalar FMAs for the
# f2v helpers and / or without the SLP vectorizer; all units without the SLP vectorizer
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V=dpe-mvs_amd/lib/variants
AB_ROUNDS=3 timeout -k 10 600 python -u tools/ab_libs.py $V/base.so $V/m_scal.so $V/m_fma.so $V/m_noslp.so $V/a_noslp.so > gpurun_out/r05ah_ab_mainscal.log 2>&1
