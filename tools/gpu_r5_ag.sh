#!/bin/bash
# round 5, call AG: packed f32 FMAs (v_pk_fma_f32) against the same operations as scalar FMAs
# (DPE_SCALAR_FMA2, SLP vectorizer off) in every kernel
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V=dpe-mvs_amd/lib/variants
AB_ROUNDS=3 timeout -k 10 400 python -u tools/ab_libs.py $V/base.so $V/scal.so > gpurun_out/r05ag_ab_scalar.log 2>&1
