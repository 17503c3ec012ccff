#!/bin/bash
# round 5, call M: weak sweep job pools over the whole workgroup (16 pixels, 256 lanes) instead of
# each wave's 4 pixels -- output check against the per-wave pools, interleaved timing, pool
# statistics, weak parity and config tests
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V=dpe-mvs_amd/lib/variants
AB_ROUNDS=4 timeout -k 10 400 python -u tools/ab_libs.py $V/wg0.so $V/wg1.so > gpurun_out/r05m_ab_wgpool.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/pool_stats.py $V/pstat_wg.so > gpurun_out/r05m_pool_stats.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_configs.py -m gpu -x -q -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/r05m_tests.log 2>&1
