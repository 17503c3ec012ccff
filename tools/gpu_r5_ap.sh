#!/bin/bash
# round 5, call AP: final validation of the build with DepthToWeak at 1 and the strong sweep at 2
# waves per workgroup
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_r5_final.sh r05ap
