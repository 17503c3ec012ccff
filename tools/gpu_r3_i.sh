#!/bin/bash
# round 3 GPU call I: bit-identity + timing A/B of the variant libraries, then the parity tests that
# exercise the weak sweep on the in-tree library
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
tag=${TAG:-r3i}
AB_ROUNDS=${AB_ROUNDS:-4} timeout -k 10 500 python -u tools/ab_libs.py "$@" > gpurun_out/${tag}_ab.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_configs.py -k "not config5_full and not config4_full" > gpurun_out/${tag}_tests.log 2>&1
