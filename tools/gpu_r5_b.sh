#!/bin/bash
# round 5, call B: v_rcp_f32 table for the oracle (tools/rcp_dump.hip) + timing A/B of the tap
# reciprocal without the Newton step (restatement choice 8) against the round-4 exact reciprocal
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 120 /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/rcp_dump.hip -o /tmp/rcp_dump || exit 1
timeout -k 10 120 /tmp/rcp_dump gpurun_out/rcp127.bin > gpurun_out/r05b_rcp_dump.log 2>&1 || exit 1
AB_NOCHECK=1 AB_ROUNDS=4 timeout -k 10 500 python -u tools/ab_libs.py dpe-mvs_amd/lib/variants/newton.so dpe-mvs_amd/lib/variants/rcp.so > gpurun_out/r05b_ab_rcp.log 2>&1
