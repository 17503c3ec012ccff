#!/bin/bash
# round 5, call AI: parity + configs on the build with the main unit's SLP vectorizer off, then the
# loop vectorizer off in every unit (A/B)
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_configs.py > gpurun_out/r05ai_parity.log 2>&1 || exit $?
V=dpe-mvs_amd/lib/variants
AB_ROUNDS=3 timeout -k 10 400 python -u tools/ab_libs.py $V/base.so $V/novec.so > gpurun_out/r05ai_ab_novec.log 2>&1
