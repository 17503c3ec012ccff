#!/bin/bash
# round 5, call O: strong sweep job pools over the whole workgroup -- output check against the
# per-wave pools, interleaved timing, pool statistics, parity and config tests
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V=dpe-mvs_amd/lib/variants
AB_ROUNDS=4 timeout -k 10 400 python -u tools/ab_libs.py $V/sg0.so $V/sg1.so $V/sg2.so > gpurun_out/r05o_ab_sgpool.log 2>&1 || exit $?

timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_configs.py -m gpu -x -q -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/r05o_tests.log 2>&1
