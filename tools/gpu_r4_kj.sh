#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_r4_k.sh && bash tools/gpu_r4_j.sh
