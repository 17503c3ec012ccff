#!/bin/bash
# round 4, call E: issue rates (with v_mad_u64_u32) and the A/B of the 64-bit-product Philox
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V=dpe-mvs_amd/lib/variants
timeout -k 10 120 tools/isa_rate > gpurun_out/r04e_isa_rate.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/ab_libs.py dpe-mvs_amd/lib/libdpe_mvs.so $V/ph64.so > gpurun_out/r04e_ab.log 2>&1
