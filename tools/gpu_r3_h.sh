#!/bin/bash
# round 3 GPU call H: timing-only A/B (outputs not compared) of variant libraries
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
AB_NOCHECK=1 AB_ROUNDS=3 timeout -k 10 500 python -u tools/ab_libs.py "$@" > gpurun_out/${TAG}_ab.log 2>&1
