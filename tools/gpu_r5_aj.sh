#!/bin/bash
# round 5, call AJ: final validation (tools/gpu_r5_final.sh) and PMC passes of the build with the
# main unit's SLP vectorizer off
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_r5_final.sh r05aj && bash tools/gpu_r5_fin_pmc.sh r05h
