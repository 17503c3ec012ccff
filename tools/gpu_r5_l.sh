#!/bin/bash
# round 5, call L: weak sweep's final candidate costs with the geometric terms over all lanes
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V=dpe-mvs_amd/lib/variants
AB_ROUNDS=4 timeout -k 10 400 python -u tools/ab_libs.py $V/fc0.so $V/fc1.so > gpurun_out/r05l_ab_fc.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r05l_parity.log 2>&1
