#!/bin/bash
# round 5, call F: weak list partitioned by centre-patch side -- results checked against the
# unpartitioned build on the bench workload, interleaved timing, weak path statistics, parity tests
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V=dpe-mvs_amd/lib/variants
AB_ROUNDS=4 timeout -k 10 400 python -u tools/ab_libs.py $V/nopart.so $V/part.so > gpurun_out/r05f_ab_part.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/weak_stats.py $V/wstat_nopart.so > gpurun_out/r05f_weak_stats.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/weak_stats.py $V/wstat_part.so >> gpurun_out/r05f_weak_stats.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r05f_parity.log 2>&1
