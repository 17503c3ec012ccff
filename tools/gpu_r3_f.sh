#!/bin/bash
# round 3 GPU call F: new GPU tests (device-hook exchange, forked schedule over pass kinds) and a
# bit-checked timing A/B of variant libraries
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
bash tools/gpu_tests_subset.sh ${TAG}_tests tests/test_resident.py tests/test_gpu_parity.py -k "device_hook or overlapped" || exit $?
AB_ROUNDS=4 timeout -k 10 500 python -u tools/ab_libs.py "$@" > gpurun_out/${TAG}_ab.log 2>&1
