#!/bin/bash
# round 4, call AG: GenEdgeInform's window counts as row + column passes (DPE_EI_SEP) -- A/B, parity
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V=dpe-mvs_amd/lib/variants
AB_ROUNDS=6 timeout -k 10 500 python -u tools/ab_libs.py dpe-mvs_amd/lib/libdpe_mvs.so $V/eisep.so > gpurun_out/r4ag_ab.log 2>&1 || exit $?
DPE_MVS_LIB=$PWD/$V/eisep.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_resident.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r4ag_parity.log 2>&1
