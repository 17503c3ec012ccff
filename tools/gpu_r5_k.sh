#!/bin/bash
# round 5, call K: weak sweep phase 1 by patch rows (tables and reference sums in one pass) -- output
# check against the previous form, interleaved timing, phase profile, weak parity tests
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V=dpe-mvs_amd/lib/variants
AB_ROUNDS=4 timeout -k 10 400 python -u tools/ab_libs.py $V/w_base.so $V/w_rows1.so > gpurun_out/r05k_ab_rows1.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/phase_prof.py $V/phase_rows1.so > gpurun_out/r05k_phase.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r05k_parity.log 2>&1
