#!/bin/bash
# round 3 GPU call A: timing A/B of the round-2 library against the round-3 tap definition
# (outputs differ by design: AB_NOCHECK), plus the raw v_rcp_f32 statistics.
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 120 bash -c '/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/rcp_check.hip -o /tmp/rcp_check && /tmp/rcp_check' > gpurun_out/r3a_rcp.log 2>&1 || exit $?
AB_NOCHECK=1 AB_ROUNDS=4 timeout -k 10 500 python -u tools/ab_libs.py "$@" > gpurun_out/r3a_ab.log 2>&1
