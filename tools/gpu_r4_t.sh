#!/bin/bash
# round 4, call T: parity of the default build (pixel-first walks, 64-bit-product Philox) and its
# bench line
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_resident.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4t_parity.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r4t_bench.log 2>&1
