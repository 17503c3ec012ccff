#!/bin/bash
# round 4, call AB2: v_rcp_f32 characterisation (tools/rcp_table.hip)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 120 tools/rcp_table > gpurun_out/r4_rcp_table.log 2>&1
