#!/bin/bash
# round 5, call T: DepthToWeak skipping selected views of zero weight (their terms are +0) -- output
# check, interleaved timing, parity + config tests
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V=dpe-mvs_amd/lib/variants
AB_ROUNDS=4 timeout -k 10 400 python -u tools/ab_libs.py $V/vw0off.so $V/vw0on.so > gpurun_out/r05t_ab_vw0.log 2>&1 || exit $?
DPE_MVS_LIB=$V/vw0on.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_configs.py -m gpu -x -q -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/r05t_tests.log 2>&1
