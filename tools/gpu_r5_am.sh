#!/bin/bash
# round 5, call AM: RandomInitialization in its own unit under max-memory-clause (the built library)
# against the same unit under the default scheduler; parity + configs on the built library
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V=dpe-mvs_amd/lib/variants
AB_ROUNDS=4 timeout -k 10 400 python -u tools/ab_libs.py $V/init_def.so dpe-mvs_amd/lib/libdpe_mvs.so > gpurun_out/r05am_ab_initsched.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_configs.py > gpurun_out/r05am_parity.log 2>&1
