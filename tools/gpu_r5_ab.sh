#!/bin/bash
# round 5, call AB: the reference patch sums once per pass (k_patch_sums) instead of per visit --
# output check, interleaved timing, parity + configs
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V=dpe-mvs_amd/lib/variants
AB_ROUNDS=4 timeout -k 10 500 python -u tools/ab_libs.py $V/ps_off.so $V/ps_on.so > gpurun_out/r05ab_ab_psum.log 2>&1 || exit $?
DPE_MVS_LIB=$V/ps_on.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_configs.py -m gpu -x -q -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/r05ab_tests.log 2>&1
