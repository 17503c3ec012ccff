#!/bin/bash
# round 3 GPU call B: gather locality of the tap kernels, and the HIP == oracle parity tests of the
# round-3 tap definition (goldens excluded).
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/line_stats.py dpe-mvs_amd/lib/variants/lstat.so > gpurun_out/r3b_lines.log 2>&1
rc=$?; echo "line_stats rc=$rc" >> gpurun_out/r3b_lines.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
tools/gpu_tests_subset.sh r3b_parity tests/test_gpu_parity.py -k "not golden"
