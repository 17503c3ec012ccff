#!/bin/bash
# round 5, call X: GenNeighbours / RANSAC draws reduced modulo the shift range / support count by a
# multiply-high quotient (tools/check_fastmod.c) -- output check, interleaved timing, parity + configs
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V=dpe-mvs_amd/lib/variants
AB_ROUNDS=5 timeout -k 10 500 python -u tools/ab_libs.py $V/fm0.so $V/fm1.so > gpurun_out/r05x_ab_fastmod.log 2>&1 || exit $?
DPE_MVS_LIB=$V/fm1.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_configs.py -m gpu -x -q -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/r05x_tests.log 2>&1
