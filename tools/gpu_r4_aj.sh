#!/bin/bash
# round 4, call AJ: the geometric term's divisions as FMA quotients (DPE_GEOM_MDIV) -- A/B against
# the IEEE-division build (outputs must be identical), then parity of the new default
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V=dpe-mvs_amd/lib/variants
AB_ROUNDS=6 timeout -k 10 500 python -u tools/ab_libs.py $V/mdiv0.so dpe-mvs_amd/lib/libdpe_mvs.so > gpurun_out/r4aj_ab.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_resident.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r4aj_parity.log 2>&1
