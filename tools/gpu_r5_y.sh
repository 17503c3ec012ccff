#!/bin/bash
# round 5, call Y: the weak sweep with the WeakTab fields as plain copies (0 B scratch) against the
# reference bindings (32 B/lane) -- output check, interleaved timing
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V=dpe-mvs_amd/lib/variants
AB_ROUNDS=5 timeout -k 10 500 python -u tools/ab_libs.py $V/tc0.so $V/tc1.so > gpurun_out/r05y_ab_tcopy.log 2>&1
