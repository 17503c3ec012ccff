#!/bin/bash
# round 3 GPU call C: HIP == oracle parity of the round-3 tap definition (goldens excluded), then a
# timing A/B of variant libraries (outputs differ from round 2 by design: AB_NOCHECK).
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
bash tools/gpu_tests_subset.sh ${TAG:-r3c}_parity tests/test_gpu_parity.py -k "not golden" || exit $?
AB_NOCHECK=1 AB_ROUNDS=4 timeout -k 10 500 python -u tools/ab_libs.py "$@" > gpurun_out/${TAG:-r3c}_ab.log 2>&1
