#!/bin/bash
# round 5, call I: GenNeighbours probes that skip the draws of steps whose targets hold no candidate
# -- results checked against the drawing build, interleaved timing, then parity + config tests
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V=dpe-mvs_amd/lib/variants
AB_ROUNDS=4 timeout -k 10 400 python -u tools/ab_libs.py $V/gn_ns0.so $V/gn_ns.so > gpurun_out/r05i_ab_gn.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_configs.py -m gpu -x -q -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/r05i_tests.log 2>&1
